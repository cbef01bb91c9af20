// tbd_tracker.hpp — native restatement of the reference's cv::tbd tracker
// (modules/trackingbydetection/include/opencv2/tbd.hpp:25-184,
//  modules/trackingbydetection/src/tbd.cpp:52-1106).
//
// The bookkeeping is bit-exact with the reference (Rect rounding, integer
// box averaging, the padded-square assignment solver with its 1e-8 zero test,
// lifecycle thresholds, the 1280x720 out-of-bounds filter), but the data
// layout is built for a per-frame hot loop: per-track history is kept as the
// bounded windows the algorithm reads (last 4 boxes, last 2 frames, last
// timeWindowSize scores) instead of ever-growing vectors, tracks are not
// copied every frame, and the cost matrix is one flat array.
//
// Track::motionModel (tbd.hpp:111) is the hook the KLT path plugs into: a
// per-track predicted centroid computed on the GPU (affine fit of the track's
// tracked corners) replaces the constant-velocity model when it is valid.
#pragma once

#include <cstdint>
#include <cstdio>
#include <map>
#include <vector>

#include "../../include/tbdk.h"

namespace tbdk {
namespace tbd {

struct Rect {
    int x = 0, y = 0, width = 0, height = 0;
    Rect() = default;
    Rect(int x_, int y_, int w_, int h_) : x(x_), y(y_), width(w_), height(h_) {}
    int area() const { return width * height; }
};

// cv::Rect(Point2d, Size): the point is converted with cvRound (round half to
// even, core/include/opencv2/core/types.hpp:1175-1178, fast_math.hpp:101-106)
Rect rect_from_point2d(double px, double py, int w, int h);

struct TbdArgs {  // cv::tbd::TbdArgs (tbd.hpp:25-41); defaults of samples/gpu/tbd.cpp:249-254
    double costOfNonAssignment = 10.0;
    unsigned timeWindowSize = 16;
    unsigned trackAgeThreshold = 4;
    double trackVisibilityThreshold = 0.3;
    double trackConfidenceThreshold = 0.2;
    bool shouldStoreMetrics = true;
    // filterTracksOutOfBounds(0, 1280, 0, 720) is hard-coded in the reference
    // (tbd.cpp:218, "TAMERT HACK" :317); kept as the default for bit-exactness
    int boundsXmin = 0, boundsXmax = 1280, boundsYmin = 0, boundsYmax = 720;
};

struct Detection {  // cv::tbd::Detection (tbd.hpp:69-83)
    int id = -1;
    int frame_id = 0;
    Rect bbox;
    double confidence = 1.0;
};

// Fixed-capacity history window: push_back drops the oldest entry when full;
// [0] is the oldest kept entry.  Trivially movable (no heap), so tracks can be
// compacted in place every frame.
template <class T, unsigned N>
struct Window {
    T v[N];
    unsigned head = 0, n = 0;
    unsigned size() const { return n; }
    void push_back(const T& x)
    {
        if (n < N) {
            v[(head + n++) % N] = x;
        } else {
            v[head] = x;
            head = (head + 1) % N;
        }
    }
    const T& operator[](unsigned k) const { return v[(head + k) % N]; }
    const T& back() const { return (*this)[n - 1]; }
};

constexpr unsigned kMaxTimeWindow = 64;  // bound on TbdArgs::timeWindowSize

struct Track {  // cv::tbd::Track (tbd.hpp:89-114) with bounded history
    unsigned id = 0;
    Window<Rect, 4> bboxes;                // last <= 4 boxes (updateAssignedTracks reads 4)
    Window<int, 2> frames;                 // last <= 2 frame ids (motion model reads 2)
    Window<double, kMaxTimeWindow> scores;  // last <= timeWindowSize scores (see push_box)
    unsigned age = 1, totalVisibleCount = 1;
    double maxConfidence = 0, avgConfidence = 0;
    Rect predPosition;
    double bboxOverlap = 1.0;
    int64_t historyLength = 1;  // number of boxes the reference vector would hold
    int color[3] = {0, 0, 0};   // display colour (tbd.cpp:71-74), drawn when the tracker has a CRand
    int slot = -1;              // GPU point-set slot (product bookkeeping, not in the reference)
};

// glibc rand()/srand() (TYPE_3 additive feedback generator, degree 31,
// separation 3; glibc stdlib/random_r.c) restated with private state.  The
// sample draws from the process-global rand(): 3 calls per new track for its
// colour (tbd.cpp:71-73) and one per frame for the history age
// (samples/gpu/tbd.cpp:660), never seeded (= srand(1)).  Keeping that
// sequence is what makes the history choices of a replay identical.
class CRand {
public:
    explicit CRand(uint32_t seed = 1) { srand(seed); }
    void srand(uint32_t seed);
    int rand();
    static constexpr int kRandMax = 2147483647;

private:
    int32_t ring[31];
    unsigned f = 3, b = 0;  // front / rear taps into the ring
};

// cv::tbd::Trajectory (tbd.hpp:46-80, tbd.cpp:119-171): the ground-truth
// history of one object and the tracking result per frame.  std::map keeps the
// reference's operator[] semantics (absent keys default-insert).
struct Trajectory {
    int id = -1;
    std::vector<int> presentFrames;
    std::map<int, Rect> positionPerFrame;
    std::map<int, bool> isTrackedPerFrame;
    std::map<int, int> trackIdPerFrame;
    std::map<int, Rect> predPosPerFrame;
    std::map<int, Rect> trackPosPerFrame;
    std::map<int, double> bboxOverlapPerFrame;
    Trajectory() = default;
    explicit Trajectory(int id_) : id(id_) {}
    void addPosition(int frame, const Rect& bbox);  // tbd.cpp:141-146 (world position: display only)
    void addTrackingInfo(int frame, const struct Track* track);  // tbd.cpp:148-171
};
using TrajectoryMap = std::map<int, Trajectory>;

// predicted centroid supplied by the KLT box propagation (per track id)
struct Prediction {
    unsigned id;
    int valid;
    double cx, cy;
};

class Tracker {
public:
    explicit Tracker(const TbdArgs& args);
    void reset();
    unsigned getNextTrackId() { return nextTrackId++; }
    std::vector<Track>& getTracks() { return tracks; }
    void setTracks(const std::vector<Track>& t) { tracks = t; }  // tbd.cpp:187-190
    // the rand() the new tracks' colours are drawn from (null: not drawn)
    void setRand(CRand* r) { rng = r; }
    // solve every frame on the dense cost matrix (the first round too); the
    // default solves the first round on the entries' value kinds (same result)
    void setDenseSolver(bool on) { denseSolver = on; }

    // Tracker::performTrackingStep (tbd.cpp:210-286).  preds (may be null)
    // override the motion model for the tracks they name.
    // traj (may be null) receives addTrackingInfo for the detections that
    // carry a ground-truth id (tbd.cpp:236-265).
    void performTrackingStep(std::vector<Detection>& dets, int frame_id, const Prediction* preds = nullptr,
                             int npreds = 0, TrajectoryMap* traj = nullptr);

    // per-frame metrics (tbd.hpp:145-151)
    std::vector<int> truePositives, falseNegatives, falsePositives, groundTruths, numMatches;
    std::vector<double> bboxOverlap;
    // product-side bookkeeping of the last step (for the GPU point sets)
    std::vector<unsigned> createdIds;  // tracks created this step
    std::vector<unsigned> deletedIds;  // tracks removed this step (filtered or lost)
    std::vector<int> lastAssignments;  // per track (after filtering), -1 unassigned
    unsigned lastRounds = 0;           // solver rounds of the last step (step 4 runs between rounds)

private:
    TbdArgs args;
    CRand* rng = nullptr;
    unsigned nextTrackId = 0;
    bool denseSolver = false;
    std::vector<Track> tracks;
    std::vector<double> cost;  // flat n x n cost matrix
    std::vector<unsigned> assignmentPerRow;
    // solver scratch, kept across frames
    std::vector<uint8_t> zero;
    std::vector<unsigned> rowZeros, colZeros, colRow, colLast, detOrder;
    std::vector<double> colMin;
    std::vector<char> rowA, colA, rowM, colM;
    std::vector<int> predIndex;
    std::vector<uint64_t> detKey;
    std::vector<int> sortedX0, sortedX1, sortedY0, sortedY1, sortedArea;
    std::vector<unsigned> cand;
    // first-round solver scratch: overlap entries per track row and per column,
    // row minima and value kinds, the zero pattern as bits
    std::vector<unsigned> exStart, exCol, colExStart, colExRow, colFill, defOrder;
    std::vector<double> exVal, exValR, colExVal, rowMinV, rowDef, rowPadV;
    std::vector<uint64_t> zbits, colAbits;

    void predictNewLocationsOfTracks(int frame_id, const Prediction* preds, int npreds);
    void filterTracksOutOfBounds(int xmin, int xmax, int ymin, int ymax);
    void solveAssignment(std::vector<Detection>& dets, std::vector<int>& assignments,
                         std::vector<unsigned>& unassignedTracks, std::vector<unsigned>& unassignedDetections);
    void updateAssignedTracks(std::vector<Detection>& dets, const std::vector<int>& assignments);
    void updateUnassignedTracks(const std::vector<unsigned>& unassignedTracks, int frame_id);
    void deleteLostTracks();
    void createNewTracks(std::vector<Detection>& dets, const std::vector<unsigned>& unassignedDetections);
    void updateTrackConfidence(Track& t);
};

double computeBoundingBoxOverlap(const Rect& a, const Rect& b);  // tbd.cpp:1085-1106

}  // namespace tbd

namespace app {  // tbd_app.cpp
// App::writeTrackingOutputToFile (samples/gpu/tbd.cpp:946-1120); path NULL/"" = metrics only
bool write_tracking_output(const tbd::Tracker& tk, const std::vector<unsigned>& historyAges,
                           tbd::TrajectoryMap& trajectoryMap, unsigned frame_count, const char* path, FILE* log,
                           tbdk_scenario_metrics* out);
// parseDetections' addPosition for every detection with a ground-truth id
void add_positions(tbd::TrajectoryMap& traj, const std::vector<tbd::Detection>& dets, int frame);
}  // namespace app

namespace tbd {

}  // namespace tbd
}  // namespace tbdk

// the host tracker behind the tbdk_tracker_* C ABI (tbd_tracker.cpp, tbd_app.cpp)
struct tbdk_tracker {
    tbdk::tbd::Tracker tracker;
    std::vector<tbdk::tbd::Detection> dets;
    std::vector<tbdk::tbd::Prediction> preds;
    explicit tbdk_tracker(const tbdk::tbd::TbdArgs& a) : tracker(a) {}
};

// std::map<int, Trajectory> behind the tbdk_trajectories C ABI (tbd_app.cpp, tbd_loop.hip)
struct tbdk_trajectories {
    tbdk::tbd::TrajectoryMap map;
};
