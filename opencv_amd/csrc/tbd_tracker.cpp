// tbd_tracker.cpp — see tbd_tracker.hpp.  Every function cites the reference
// function (modules/trackingbydetection/src/tbd.cpp) whose behaviour it restates.
#include "tbd_tracker.hpp"

#include <cstring>
#include <new>

#include "../../include/tbdk.h"

#include <algorithm>
#include <cmath>
#if defined(__SSE2__)
#include <emmintrin.h>
#endif
#include <cstdint>

namespace tbdk {
namespace tbd {

Rect rect_from_point2d(double px, double py, int w, int h)
{
    // saturate_cast<int>(double) == cvRound: nearbyint under the default
    // round-to-nearest-even mode (fast_math.hpp:101-106, _mm_cvtsd_si32)
    return Rect((int)std::nearbyint(px), (int)std::nearbyint(py), w, h);
}

double computeBoundingBoxOverlap(const Rect& a, const Rect& b)
{
    const double xleft = std::max(a.x, b.x);
    const double xright = std::min(a.x + a.width, b.x + b.width);
    const double ytop = std::max(a.y, b.y);
    const double ybottom = std::min(a.y + a.height, b.y + b.height);
    if ((xright < xleft) || (ybottom < ytop)) return 0.0;
    const double inter = (xright - xleft) * (ybottom - ytop);
    const double uni = a.area() + b.area() - inter;
    return inter / uni;
}

static inline bool equalsZero(double v)  // tbd.hpp:178-181
{
    return (v < 0.0) ? (v > -0.00000001) : (v < 0.00000001);
}

// srandom_r / random_r, TYPE_3 (glibc stdlib/random_r.c)
void CRand::srand(uint32_t seed)
{
    if (seed == 0) seed = 1;
    int32_t word = (int32_t)seed;
    ring[0] = word;
    for (int i = 1; i < 31; ++i) {
        // 16807 * word % 2147483647 without overflow (Schrage)
        const long hi = word / 127773, lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        ring[i] = word;
    }
    f = 3;
    b = 0;
    for (int i = 0; i < 310; ++i) rand();
}

int CRand::rand()
{
    const uint32_t val = (uint32_t)ring[f] + (uint32_t)ring[b];
    ring[f] = (int32_t)val;
    if (++f >= 31) {
        f = 0;
        ++b;
    } else if (++b >= 31) {
        b = 0;
    }
    return (int)(val >> 1);
}

void Trajectory::addPosition(int frame, const Rect& bbox)
{
    presentFrames.push_back(frame);
    positionPerFrame[frame] = bbox;
}

void Trajectory::addTrackingInfo(int frame, const Track* track)
{
    if (track) {
        isTrackedPerFrame[frame] = true;
        trackIdPerFrame[frame] = (int)track->id;
        const Rect& bbox = track->bboxes.back();
        const Rect& gt = positionPerFrame[frame];  // default-inserted if absent, as map::operator[]
        trackPosPerFrame[frame] = bbox;
        predPosPerFrame[frame] = track->predPosition;
        bboxOverlapPerFrame[frame] = computeBoundingBoxOverlap(bbox, gt);
    } else {
        isTrackedPerFrame[frame] = false;
    }
}

Tracker::Tracker(const TbdArgs& a) : args(a) {}

void Tracker::reset()  // tbd.cpp:197-208
{
    nextTrackId = 0;
    tracks.clear();
    truePositives.clear();
    falseNegatives.clear();
    falsePositives.clear();
    groundTruths.clear();
    numMatches.clear();
    bboxOverlap.clear();
}

// constantVelocityMotionModel (tbd.cpp:1057-1083)
static void constant_velocity(const Track& t, int frame_id, double& cx, double& cy)
{
    if (t.age == 1) {
        const Rect& b = t.bboxes.back();
        cx = b.x + b.width / 2;
        cy = b.y + b.height / 2;
        return;
    }
    const int f1 = t.frames[t.frames.size() - 1], f2 = t.frames[t.frames.size() - 2];
    const Rect& b1 = t.bboxes[t.bboxes.size() - 1];
    const Rect& b2 = t.bboxes[t.bboxes.size() - 2];
    const double ratio = ((double)(frame_id - f1)) / (f1 - f2);
    const double dx = ratio * (b1.x - b2.x);
    const double dy = ratio * (b1.y - b2.y);
    const double w = (b1.width + b2.width) / 2.0;
    const double h = (b1.height + b2.height) / 2.0;
    cx = b1.x + w / 2 + dx;
    cy = b1.y + h / 2 + dy;
}

// predictNewLocationsOfTracks (tbd.cpp:288-304) with the KLT hook
void Tracker::predictNewLocationsOfTracks(int frame_id, const Prediction* preds, int npreds)
{
    // first valid prediction per id, looked up by binary search
    predIndex.clear();
    for (int k = 0; preds && k < npreds; ++k)
        if (preds[k].valid) predIndex.push_back(k);
    std::stable_sort(predIndex.begin(), predIndex.end(),
                     [&](int a, int b) { return preds[a].id < preds[b].id; });
    for (auto& t : tracks) {
        const Rect& bbox = t.bboxes.back();
        double cx, cy;
        const Prediction* p = nullptr;
        auto it = std::lower_bound(predIndex.begin(), predIndex.end(), t.id,
                                   [&](int k, unsigned id) { return preds[k].id < id; });
        if (it != predIndex.end() && preds[*it].id == t.id) p = &preds[*it];
        if (p) {
            cx = p->cx;
            cy = p->cy;
        } else {
            constant_velocity(t, frame_id, cx, cy);
        }
        t.predPosition = rect_from_point2d(cx - bbox.width / 2, cy - bbox.height / 2, bbox.width, bbox.height);
    }
}

// filterTracksOutOfBounds (tbd.cpp:306-331)
void Tracker::filterTracksOutOfBounds(int xmin, int xmax, int ymin, int ymax)
{
    size_t k = 0;
    for (size_t i = 0; i < tracks.size(); ++i) {
        const Rect& r = tracks[i].predPosition;
        if (r.x + r.width < xmin || r.x >= xmax || r.y + r.height < ymin || r.y >= ymax)
            deletedIds.push_back(tracks[i].id);
        else if (k++ != i)
            tracks[k - 1] = tracks[i];
    }
    tracks.resize(k);
}

// min over a row with the reference's `(v < m) ? v : m` step.  The value does
// not depend on the scan order (a NaN is never selected by `<`), so it is
// taken two lanes at a time: MINPD(v, m) is exactly (v < m) ? v : m per lane.
static double row_min(const double* row, unsigned n, double init)
{
    unsigned c = 0;
    double m = init;
#if defined(__SSE2__)
    __m128d a = _mm_set1_pd(init), b = _mm_set1_pd(init);
    for (; c + 4 <= n; c += 4) {
        a = _mm_min_pd(_mm_loadu_pd(row + c), a);
        b = _mm_min_pd(_mm_loadu_pd(row + c + 2), b);
    }
    a = _mm_min_pd(b, a);
    double t[2];
    _mm_storeu_pd(t, a);
    m = (t[1] < t[0]) ? t[1] : t[0];
#endif
    for (; c < n; ++c) m = (row[c] < m) ? row[c] : m;
    return m;
}

// The dense passes of the solver, built for AVX2 and baseline x86-64 (picked
// at load time).  Elementwise IEEE operations only (no contraction: the file is
// built with -ffp-contract=off), so every value is the same in both builds.
#define TBDK_SOLVER_CLONES __attribute__((target_clones("avx2", "default")))

// row -= m (step 1, :507-516), fused with step 2's running column minima
// (:539-561, rows in order): colMin[c] = (row[c] < colMin[c]) ? row[c] : colMin[c]
TBDK_SOLVER_CLONES static void sub_row_min_and_colmin(double* __restrict row, unsigned n, double m,
                                                      double* __restrict colMin)
{
    for (unsigned c = 0; c < n; ++c) {
        const double v = row[c] - m;
        row[c] = v;
        colMin[c] = (v < colMin[c]) ? v : colMin[c];
    }
}

// one row of the zero pattern (equalsZero, tbd.hpp:178-181), optionally after
// subtracting the column minima (step 2); returns the row's zero count and
// adds the row to the column counts and "last zero row" of every column
TBDK_SOLVER_CLONES static unsigned zero_row(double* __restrict row, const double* __restrict colMin, unsigned n,
                                           uint8_t* __restrict z, unsigned* __restrict colZeros,
                                           unsigned* __restrict colLast, unsigned r)
{
    if (colMin)
        for (unsigned c = 0; c < n; ++c) row[c] -= colMin[c];
    unsigned cnt = 0;
    for (unsigned c = 0; c < n; ++c) {
        const uint8_t v = std::fabs(row[c]) < 0.00000001 ? 1 : 0;
        z[c] = v;
        cnt += v;
    }
    if (cnt)
        for (unsigned c = 0; c < n; ++c) {
            colZeros[c] += z[c];
            colLast[c] = z[c] ? r : colLast[c];  // row of a column's single zero
        }
    return cnt;
}

// calculateCostMatrix + solveAssignmentProblem + classifyAssignments
// (tbd.cpp:333-891) on a flat n x n matrix.  The reference's operation order
// on every matrix entry is kept (row minima, column minima, the step-4
// subtract/add of mu), so every comparison sees the same doubles; only the
// loop nests are reorganised for the cache and the vector units: column
// minima are accumulated row by row (same r order per column), the zero
// pattern and its row/column counts are rebuilt in one pass, and the
// "row assigned to column c" lookup of the cover step is an inverse map.
void Tracker::solveAssignment(std::vector<Detection>& dets, std::vector<int>& assignments,
                              std::vector<unsigned>& unassignedTracks, std::vector<unsigned>& unassignedDetections)
{
    const unsigned nT = (unsigned)tracks.size(), nD = (unsigned)dets.size();
    const unsigned n = std::max(nT, nD);
    const double huge = 10000000.0;
    const double pad = args.costOfNonAssignment * 2;
    cost.resize((size_t)n * n);
    detX0.resize(nD); detY0.resize(nD); detX1.resize(nD); detY1.resize(nD); detArea.resize(nD);
    detOrder.resize(nD);
    int maxW = 0;
    for (unsigned j = 0; j < nD; ++j) {
        const Rect& b = dets[j].bbox;
        detX0[j] = b.x; detY0[j] = b.y; detX1[j] = b.x + b.width; detY1[j] = b.y + b.height;
        detArea[j] = b.area();
        detOrder[j] = j;
        maxW = std::max(maxW, b.width);
    }
    // detections by left edge: a track row only visits the detections whose x-range
    // can touch its box; all others are strictly separated, where the reference's
    // computeBoundingBoxOverlap returns exactly 0.0 (cost exactly 1.0)
    std::sort(detOrder.begin(), detOrder.end(), [&](unsigned a, unsigned b) { return detX0[a] < detX0[b]; });
    sortedX0.resize(nD);
    for (unsigned k = 0; k < nD; ++k) sortedX0[k] = detX0[detOrder[k]];
    assignmentPerRow.assign(n, n);
    if (n == 0) return;
    colMin.assign(n, huge);
    // calculateCostMatrix (:333-351) fused with step 1, the row minima (:494-516),
    // and step 2's column minima
    for (unsigned r = 0; r < n; ++r) {
        double* row = &cost[(size_t)r * n];
        unsigned c0 = 0;
        if (r < nT) {
            const Rect& p = tracks[r].predPosition;
            const int px0 = p.x, py0 = p.y, px1 = p.x + p.width, py1 = p.y + p.height, pa = p.area();
            for (unsigned j = 0; j < nD; ++j) row[j] = 1.0;
            const unsigned lb = (unsigned)(std::lower_bound(sortedX0.begin(), sortedX0.end(), px0 - maxW) -
                                           sortedX0.begin());
            const unsigned ub = (unsigned)(std::upper_bound(sortedX0.begin(), sortedX0.end(), px1) - sortedX0.begin());
            for (unsigned k = lb; k < ub; ++k) {
                const unsigned j = detOrder[k];
                if (detX0[j] > px1 || detX1[j] < px0 || detY0[j] > py1 || detY1[j] < py0) continue;
                const int xl = std::max(px0, detX0[j]), xr = std::min(px1, detX1[j]);
                const int yt = std::max(py0, detY0[j]), yb = std::min(py1, detY1[j]);
                if (xr < xl || yb < yt) continue;  // (:1094-1097) -> 0.0
                const double inter = (double)(xr - xl) * (double)(yb - yt);
                const double uni = (double)(pa + detArea[j]) - inter;
                row[j] = 1.0 - inter / uni;
            }
            c0 = nD;
        }
        for (unsigned c = c0; c < n; ++c) row[c] = pad;
        sub_row_min_and_colmin(row, n, row_min(row, n, huge), colMin.data());
    }
    {
        // the column minima's subtraction is fused into the first round's zero pass
        zero.resize((size_t)n * n);
        rowZeros.resize(n);
        colZeros.resize(n);
        colLast.resize(n);
        colRow.resize(n);
        rowA.resize(n);
        colA.resize(n);
        rowM.resize(n);
        colM.resize(n);
        bool first = true;
        while (true) {  // (:585-887)
            std::fill(colZeros.begin(), colZeros.end(), 0u);
            for (unsigned r = 0; r < n; ++r)
                rowZeros[r] = zero_row(&cost[(size_t)r * n], first ? colMin.data() : nullptr, n, &zero[(size_t)r * n],
                                       colZeros.data(), colLast.data(), r);
            first = false;
            std::fill(rowA.begin(), rowA.end(), 0);
            std::fill(colA.begin(), colA.end(), 0);
            std::fill(colRow.begin(), colRow.end(), n);
            unsigned numAssigned = 0;
            assignmentPerRow.assign(n, n);
            auto assign = [&](unsigned r, unsigned c) {
                rowA[r] = colA[c] = 1;
                assignmentPerRow[r] = c;
                colRow[c] = r;
                numAssigned++;
            };
            bool made = true;
            while (made) {
                made = false;
                // rows with exactly one zero (:607-636)
                for (unsigned r = 0; r < n; ++r) {
                    if (rowA[r] || rowZeros[r] != 1) continue;
                    const uint8_t* z = &zero[(size_t)r * n];
                    unsigned c = 0;
                    while (!z[c]) ++c;
                    if (!colA[c]) {
                        assign(r, c);
                        made = true;
                    }
                }
                // columns with exactly one zero (:639-668)
                for (unsigned c = 0; c < n; ++c) {
                    if (colA[c] || colZeros[c] != 1) continue;
                    const unsigned r = colLast[c];
                    if (!rowA[r]) {
                        assign(r, c);
                        made = true;
                    }
                }
                // otherwise: first free zero of every unassigned row (:672-714)
                if (!made) {
                    for (unsigned r = 0; r < n; ++r) {
                        if (rowA[r]) continue;
                        const uint8_t* z = &zero[(size_t)r * n];
                        for (unsigned c = 0; c < n; ++c) {
                            if (z[c] && !colA[c]) {
                                assign(r, c);
                                made = true;
                                break;
                            }
                        }
                    }
                }
            }
            if (numAssigned == n) break;
            // step 3: cover zeros (:735-829)
            for (unsigned r = 0; r < n; ++r) rowM[r] = !rowA[r];
            std::fill(colM.begin(), colM.end(), 0);
            while (true) {
                unsigned newly = 0;
                for (unsigned r = 0; r < n; ++r) {
                    if (!rowM[r]) continue;
                    const uint8_t* z = &zero[(size_t)r * n];
                    for (unsigned c = 0; c < n; ++c)
                        if (z[c] && !colM[c]) {
                            colM[c] = 1;
                            newly++;
                        }
                }
                for (unsigned c = 0; c < n; ++c)
                    if (colM[c] && colRow[c] < n) rowM[colRow[c]] = 1;
                if (newly == 0) break;
            }
            bool allMarked = true;
            for (unsigned r = 0; r < n; ++r)
                if (!rowM[r]) allMarked = false;
            if (allMarked) break;
            // step 4 (:853-886): covered rows are the unmarked ones, covered columns the marked ones
            double mu = huge;
            for (unsigned r = 0; r < n; ++r) {
                if (!rowM[r]) continue;
                const double* row = &cost[(size_t)r * n];
                for (unsigned c = 0; c < n; ++c) {
                    if (colM[c]) continue;
                    mu = (row[c] < mu) ? row[c] : mu;
                }
            }
            for (unsigned r = 0; r < n; ++r) {
                double* row = &cost[(size_t)r * n];
                if (rowM[r]) {
                    for (unsigned c = 0; c < n; ++c)
                        if (!colM[c]) row[c] -= mu;
                } else {
                    for (unsigned c = 0; c < n; ++c)
                        if (colM[c]) row[c] += mu;
                }
            }
        }
    }
    // classifyAssignments (:353-379)
    std::vector<char> detA(nD, 0);
    for (unsigned i = 0; i < nT; ++i) {
        if (assignmentPerRow[i] < nD) {
            assignments.push_back((int)assignmentPerRow[i]);
            detA[assignmentPerRow[i]] = 1;
        } else {
            assignments.push_back(-1);
            unassignedTracks.push_back(i);
        }
    }
    for (unsigned j = 0; j < nD; ++j)
        if (!detA[j]) unassignedDetections.push_back(j);
}

// updateTrackConfidence (tbd.cpp:913-930)
void Tracker::updateTrackConfidence(Track& t)
{
    const unsigned num = (unsigned)t.scores.size() < args.timeWindowSize ? (unsigned)t.scores.size()
                                                                          : args.timeWindowSize;
    double maxScore = 0.0, sum = 0.0;
    for (unsigned k = t.scores.size() - num; k < t.scores.size(); ++k) {
        const double s = t.scores[k];
        sum += s;
        if (s > maxScore) maxScore = s;
    }
    t.maxConfidence = maxScore;
    t.avgConfidence = sum / num;
}

// the windows keep at least what the reference reads of its ever-growing
// vectors: 4 boxes, 2 frame ids, timeWindowSize (<= kMaxTimeWindow) scores
static void push_box(Track& t, const Rect& r, int frame, double score)
{
    t.bboxes.push_back(r);
    t.frames.push_back(frame);
    t.scores.push_back(score);
    t.historyLength++;
}

// updateAssignedTracks (tbd.cpp:935-981)
void Tracker::updateAssignedTracks(std::vector<Detection>& dets, const std::vector<int>& assignments)
{
    for (size_t i = 0; i < tracks.size(); ++i) {
        if (assignments[i] < 0) continue;
        Track& t = tracks[i];
        const Detection& d = dets[(size_t)assignments[i]];
        const unsigned nprior = t.historyLength < 4 ? (unsigned)t.historyLength : 4u;
        unsigned wsum = 0, hsum = 0;
        for (unsigned k = t.bboxes.size() - nprior; k < t.bboxes.size(); ++k) {
            wsum += t.bboxes[k].width;
            hsum += t.bboxes[k].height;
        }
        const int w = (wsum + d.bbox.width) / (nprior + 1);
        const int h = (hsum + d.bbox.height) / (nprior + 1);
        double cx = d.bbox.x, cy = d.bbox.y;
        cx += (d.bbox.width / 2) - (w / 2);
        cy += (d.bbox.height / 2) - (h / 2);
        t.bboxOverlap = computeBoundingBoxOverlap(d.bbox, t.predPosition);
        push_box(t, rect_from_point2d(cx, cy, w, h), d.frame_id, d.confidence);
        t.age++;
        t.totalVisibleCount++;
        updateTrackConfidence(t);
    }
}

// updateUnassignedTracks (tbd.cpp:986-1009)
void Tracker::updateUnassignedTracks(const std::vector<unsigned>& un, int frame_id)
{
    for (unsigned idx : un) {
        Track& t = tracks[idx];
        t.age++;
        push_box(t, t.predPosition, frame_id, 0.0);
        t.bboxOverlap = 0.0;
        updateTrackConfidence(t);
    }
}

// deleteLostTracks (tbd.cpp:1011-1037)
void Tracker::deleteLostTracks()
{
    size_t k = 0;
    for (size_t i = 0; i < tracks.size(); ++i) {
        const Track& t = tracks[i];
        const double visibility = ((double)t.totalVisibleCount) / t.age;
        if ((t.age <= args.trackAgeThreshold && visibility <= args.trackVisibilityThreshold) ||
            (t.maxConfidence >= 0.0 && t.maxConfidence <= args.trackConfidenceThreshold))
            deletedIds.push_back(t.id);
        else if (k++ != i)
            tracks[k - 1] = tracks[i];
    }
    tracks.resize(k);
}

// createNewTracks + Track::Track(Detection&, Tracker*) (tbd.cpp:1043-1055, 67-91);
// the display colour is drawn from the attached CRand (rand() % 256 x 3, :71-74)
void Tracker::createNewTracks(std::vector<Detection>& dets, const std::vector<unsigned>& un)
{
    for (unsigned j : un) {
        const Detection& d = dets[j];
        Track t;
        t.id = getNextTrackId();
        t.bboxes.push_back(d.bbox);
        t.scores.push_back(d.confidence);
        t.frames.push_back(d.frame_id);
        t.age = 1;
        t.totalVisibleCount = 1;
        t.maxConfidence = d.confidence;
        t.avgConfidence = d.confidence;
        t.predPosition = d.bbox;
        t.bboxOverlap = 1.0;
        t.historyLength = 1;
        if (rng)
            for (int c = 0; c < 3; ++c) t.color[c] = rng->rand() % 256;
        createdIds.push_back(t.id);
        tracks.push_back(std::move(t));
    }
}

// performTrackingStep (tbd.cpp:210-286)
void Tracker::performTrackingStep(std::vector<Detection>& dets, int frame_id, const Prediction* preds, int npreds,
                                  TrajectoryMap* traj)
{
    createdIds.clear();
    deletedIds.clear();
    predictNewLocationsOfTracks(frame_id, preds, npreds);
    filterTracksOutOfBounds(args.boundsXmin, args.boundsXmax, args.boundsYmin, args.boundsYmax);
    std::vector<int> assignments;
    std::vector<unsigned> unassignedTracks, unassignedDetections;
    solveAssignment(dets, assignments, unassignedTracks, unassignedDetections);
    updateAssignedTracks(dets, assignments);
    updateUnassignedTracks(unassignedTracks, frame_id);
    unsigned numAssigned = 0;
    for (size_t i = 0; i < tracks.size(); ++i) {
        if (assignments[i] < 0) continue;
        numAssigned++;
        const Detection& d = dets[(size_t)assignments[i]];
        if (traj && d.id >= 0) (*traj)[d.id].addTrackingInfo(frame_id, &tracks[i]);
    }
    // unassigned detections: the tracks created for them below are not recorded (tbd.cpp:255-265)
    if (traj)
        for (unsigned j : unassignedDetections)
            if (dets[j].id >= 0) (*traj)[dets[j].id].addTrackingInfo(frame_id, nullptr);
    lastAssignments = assignments;
    deleteLostTracks();
    createNewTracks(dets, unassignedDetections);
    if (args.shouldStoreMetrics) {
        truePositives.push_back((int)numAssigned);
        falseNegatives.push_back((int)unassignedDetections.size());
        falsePositives.push_back((int)unassignedTracks.size());
        groundTruths.push_back((int)dets.size());
        numMatches.push_back((int)numAssigned);
        double ov = 0.0;
        for (auto& t : tracks) ov += t.bboxOverlap;
        bboxOverlap.push_back(ov);
    }
}

}  // namespace tbd
}  // namespace tbdk

// ---- host-only C ABI of the tracker (include/tbdk.h) ----

extern "C" {

int tbdk_tracker_default_args(tbdk_tracker_args* a)
{
    if (!a) return TBDK_EINVAL;
    const tbdk::tbd::TbdArgs d;
    a->cost_of_non_assignment = d.costOfNonAssignment;
    a->time_window_size = (int32_t)d.timeWindowSize;
    a->track_age_threshold = (int32_t)d.trackAgeThreshold;
    a->track_visibility_threshold = d.trackVisibilityThreshold;
    a->track_confidence_threshold = d.trackConfidenceThreshold;
    a->bounds_xmin = d.boundsXmin;
    a->bounds_xmax = d.boundsXmax;
    a->bounds_ymin = d.boundsYmin;
    a->bounds_ymax = d.boundsYmax;
    return TBDK_OK;
}

int tbdk_tracker_create(const tbdk_tracker_args* a, tbdk_tracker** out)
{
    if (!a || !out || a->time_window_size <= 0 || a->time_window_size > (int)tbdk::tbd::kMaxTimeWindow ||
        a->track_age_threshold < 0)
        return TBDK_EINVAL;
    tbdk::tbd::TbdArgs t;
    t.costOfNonAssignment = a->cost_of_non_assignment;
    t.timeWindowSize = (unsigned)a->time_window_size;
    t.trackAgeThreshold = (unsigned)a->track_age_threshold;
    t.trackVisibilityThreshold = a->track_visibility_threshold;
    t.trackConfidenceThreshold = a->track_confidence_threshold;
    t.boundsXmin = a->bounds_xmin;
    t.boundsXmax = a->bounds_xmax;
    t.boundsYmin = a->bounds_ymin;
    t.boundsYmax = a->bounds_ymax;
    *out = new (std::nothrow) tbdk_tracker(t);
    return *out ? TBDK_OK : TBDK_ENOMEM;
}

int tbdk_tracker_destroy(tbdk_tracker* t)
{
    if (!t) return TBDK_EINVAL;
    delete t;
    return TBDK_OK;
}

int tbdk_tracker_step(tbdk_tracker* t, const tbdk_detection* dets, int ndets, int frame_id,
                      const tbdk_prediction* preds, int npreds, tbdk_frame_metrics* m)
{
    if (!t || ndets < 0 || (ndets > 0 && !dets) || npreds < 0 || (npreds > 0 && !preds)) return TBDK_EINVAL;
    t->dets.resize((size_t)ndets);
    for (int i = 0; i < ndets; ++i) {
        tbdk::tbd::Detection& d = t->dets[(size_t)i];
        d.id = dets[i].id;
        d.frame_id = frame_id;
        d.bbox = tbdk::tbd::Rect(dets[i].x, dets[i].y, dets[i].width, dets[i].height);
        d.confidence = dets[i].confidence;
    }
    t->preds.resize((size_t)npreds);
    for (int i = 0; i < npreds; ++i)
        t->preds[(size_t)i] = tbdk::tbd::Prediction{preds[i].track_id, preds[i].valid, preds[i].cx, preds[i].cy};
    t->tracker.performTrackingStep(t->dets, frame_id, t->preds.data(), npreds);
    if (m) {
        std::memset(m, 0, sizeof(*m));
        const tbdk::tbd::Tracker& k = t->tracker;
        m->tp = k.truePositives.back();
        m->fn = k.falseNegatives.back();
        m->fp = k.falsePositives.back();
        m->gt = k.groundTruths.back();
        m->matches = k.numMatches.back();
        m->bbox_overlap = k.bboxOverlap.back();
        m->ntracks = (int32_t)t->tracker.getTracks().size();
    }
    return TBDK_OK;
}

int tbdk_tracker_tracks(const tbdk_tracker* t, tbdk_track_info* out, int cap, int* n)
{
    if (!t || !n || cap < 0 || (cap > 0 && !out)) return TBDK_EINVAL;
    const auto& tracks = const_cast<tbdk_tracker*>(t)->tracker.getTracks();
    int k = 0;
    for (const auto& tr : tracks) {
        if (k >= cap) break;
        tbdk_track_info& o = out[k++];
        const tbdk::tbd::Rect& b = tr.bboxes.back();
        o.id = tr.id;
        o.x = b.x;
        o.y = b.y;
        o.width = b.width;
        o.height = b.height;
        o.pred_x = tr.predPosition.x;
        o.pred_y = tr.predPosition.y;
        o.pred_w = tr.predPosition.width;
        o.pred_h = tr.predPosition.height;
        o.age = (int32_t)tr.age;
        o.total_visible = (int32_t)tr.totalVisibleCount;
        o.npoints = 0;
        o.max_confidence = tr.maxConfidence;
        o.bbox_overlap = tr.bboxOverlap;
    }
    *n = (int)tracks.size();
    return TBDK_OK;
}

}  // extern "C"
