// tbd_app.cpp — the tracking driver of the reference sample
// (samples/gpu/tbd.cpp) restated natively around the tbdk tracker:
//
//   parseBboxFile                  samples/gpu/tbd.cpp:1163-1295
//   parseDetections                samples/gpu/tbd.cpp:1297-1340
//   Args::parseHistoryDistribution samples/gpu/tbd.cpp:258-291
//   App::run (tracking section)    samples/gpu/tbd.cpp:479-706, 823-841
//   App::writeTrackingOutputToFile samples/gpu/tbd.cpp:946-1120
//
// Host only (no device work): the sample feeds the tracker ground-truth or
// external detections from a bbox file; the image path (HOG, drawing, video
// I/O) is outside this library.  Every quirk that reaches the outputs is kept:
// the substr(prev_pos, pos) field parsing (a prefix parse of the field), the
// frame-offset rule (ground-truth files start at their first frame, detection
// files at 0), the dropped last frame when the file runs past num_frames, the
// float arithmetic of the history draw, the "isNew" lag of the ID-switch scan,
// default-inserting map lookups and the iostream formatting (%g, 6 digits).
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <new>
#include <string>
#include <vector>

#include "../../include/tbdk.h"
#include "tbd_tracker.hpp"

namespace tbdk {
namespace app {

using tbd::Rect;

// ---- std::stoi / stoul / stod / stof (prefix parses; throw -> false) ----
static bool c_stoi(const char* s, int& out)
{
    char* end;
    errno = 0;
    const long v = std::strtol(s, &end, 10);
    if (end == s || errno == ERANGE || v < INT_MIN || v > INT_MAX) return false;
    out = (int)v;
    return true;
}

static bool c_stoul(const char* s, unsigned long& out)
{
    char* end;
    errno = 0;
    const unsigned long v = std::strtoul(s, &end, 10);
    if (end == s || errno == ERANGE) return false;
    out = v;
    return true;
}

static bool c_stod(const char* s, double& out)
{
    char* end;
    errno = 0;
    const double v = std::strtod(s, &end);
    if (end == s || errno == ERANGE) return false;
    out = v;
    return true;
}

static bool c_stof(const char* s, float& out)
{
    char* end;
    errno = 0;
    const float v = std::strtof(s, &end);
    if (end == s || errno == ERANGE) return false;
    out = v;
    return true;
}

// one parsed bbox file: per frame, rows {objId, v1, v2, ...} (parseBboxFile's
// vector<vector<vector<double>>>)
struct BboxTable {
    std::vector<std::vector<std::vector<double>>> frames;
};

}  // namespace app
}  // namespace tbdk

using tbdk::app::BboxTable;
using tbdk::tbd::Rect;

struct tbdk_sequence {
    BboxTable cls[2];                          // 0 pedestrians, 1 vehicles
    std::vector<std::vector<double>> poses;    // per_frame_camera_poses (shared)
    std::vector<unsigned> history;             // per_frame_history_choices (shared)
    std::string error;
};

struct tbdk_track_buffer {
    std::vector<std::vector<tbdk::tbd::Track>> slots;
};

struct tbdk_rand {
    tbdk::tbd::CRand r;
    explicit tbdk_rand(uint32_t seed) : r(seed) {}
};


namespace tbdk {
namespace app {

// parseBboxFile (samples/gpu/tbd.cpp:1163-1295).  Returns false where the
// reference's stoi/stoul/stod would throw (the sample then exits "error: ...").
static bool parse_bbox_file(const char* path, unsigned num_frames, BboxTable& table,
                            std::vector<std::vector<double>>& poses, std::vector<unsigned>& history,
                            std::string& err)
{
    const bool parsePoses = poses.empty();
    FILE* f = std::fopen(path, "rb");
    // an unopenable ifstream reads no lines: the table is num_frames empty frames
    std::string line;
    int prev_frame = -1, start_frame = -1;
    std::vector<std::vector<double>> cur;
    auto& per_frame = table.frames;
    auto fail = [&](const char* what) {
        err = std::string("bbox file ") + path + ": " + what + " in line: " + line;
        if (f) std::fclose(f);
        return false;
    };
    while (f) {
        // std::getline: up to '\n' (excluded); a last line without '\n' counts
        line.clear();
        int c;
        bool got = false;
        while ((c = std::fgetc(f)) != EOF) {
            got = true;
            if (c == '\n') break;
            line.push_back((char)c);
        }
        if (!got) break;
        size_t pos = line.find('|');
        if (pos == std::string::npos) continue;
        size_t prev_pos;
        if (history.empty() && line.find("history") != std::string::npos) {
            prev_pos = pos + 1;
            do {
                pos = line.find(',', prev_pos);
                unsigned long v;
                if (!c_stoul(line.c_str() + std::min(prev_pos, line.size()), v)) return fail("stoul");
                history.push_back((unsigned)(int)v);
                prev_pos = pos + 1;
            } while (pos != std::string::npos);
            continue;
        }
        prev_pos = pos + 1;
        int frame_num;
        // stoi(line.substr(0, pos)): the field alone
        if (!c_stoi(line.substr(0, pos).c_str(), frame_num)) return fail("stoi");
        const size_t nseps = (size_t)std::count(line.begin(), line.end(), '|');
        const bool is_gt = nseps > 4;
        if (start_frame == -1) {
            start_frame = is_gt ? frame_num : 0;
            prev_frame = start_frame;
        }
        for (int i = prev_frame; i < frame_num; ++i) {
            per_frame.push_back(cur);
            cur.clear();
        }
        int objId;
        if (!is_gt) {
            objId = -2;
        } else {
            pos = line.find('|', prev_pos);
            if (!c_stoi(line.c_str() + prev_pos, objId)) return fail("stoi");
            prev_pos = pos + 1;
        }
        if (parsePoses && objId == -1) {
            std::vector<double> pose;
            do {
                pos = line.find('|', prev_pos);
                double v;
                if (prev_pos > line.size() || !c_stod(line.c_str() + prev_pos, v)) return fail("stod");
                pose.push_back(v);
                prev_pos = pos + 1;
            } while (pos != std::string::npos);
            poses.push_back(pose);
        } else if (objId != -1) {
            std::vector<double> info;
            info.push_back(objId);
            do {
                pos = line.find('|', prev_pos);
                double v;
                if (prev_pos > line.size() || !c_stod(line.c_str() + prev_pos, v)) return fail("stod");
                info.push_back(v);
                prev_pos = pos + 1;
            } while (pos != std::string::npos);
            cur.push_back(info);
        }
        prev_frame = frame_num;
    }
    if (f) std::fclose(f);
    // int i < (start_frame + unsigned num_frames): compared as unsigned, so an
    // empty file (start -1) adds nothing
    for (int i = prev_frame; (unsigned)i < (unsigned)start_frame + num_frames; ++i) {
        per_frame.push_back(cur);
        cur.clear();
    }
    return true;
}

// double -> int as the reference's implicit conversions (truncation; x86
// cvttsd2si gives INT_MIN out of range)
static inline int d2i(double v)
{
    if (!(v > -2147483649.0 && v < 2147483648.0)) return INT_MIN;
    return (int)v;
}

// parseDetections (samples/gpu/tbd.cpp:1297-1340)
static void parse_detections(const BboxTable& table, int frame, std::vector<tbd::Detection>& out,
                             tbd::TrajectoryMap* traj)
{
    out.clear();
    if (table.frames.empty() || frame < 0 || (size_t)frame >= table.frames.size()) return;
    for (const auto& b : table.frames[(size_t)frame]) {
        tbd::Detection d;
        d.id = d2i(b[0]);
        d.frame_id = frame;
        // Rect(bbox[1], bbox[3], bbox[2] - bbox[1], bbox[4] - bbox[3]): Rect_<int>
        // from doubles, each argument truncated (sizes after the subtraction)
        const double v1 = b.size() > 1 ? b[1] : 0, v2 = b.size() > 2 ? b[2] : 0;
        const double v3 = b.size() > 3 ? b[3] : 0, v4 = b.size() > 4 ? b[4] : 0;
        d.bbox = Rect(d2i(v1), d2i(v3), d2i(v2 - v1), d2i(v4 - v3));
        d.confidence = 1.0;
        out.push_back(d);
        if (d.id >= 0 && traj) {
            auto it = traj->find(d.id);
            if (it == traj->end()) it = traj->emplace(d.id, tbd::Trajectory(d.id)).first;
            it->second.addPosition(frame, d.bbox);
        }
    }
}

// Args::parseHistoryDistribution (samples/gpu/tbd.cpp:258-291)
static bool parse_history_distribution(const char* s, std::vector<float>& dist)
{
    dist.clear();
    const std::string str(s);
    size_t prev_pos = 0, pos;
    do {
        pos = str.find(',', prev_pos);
        float v;
        if (prev_pos > str.size() || !c_stof(str.c_str() + prev_pos, v)) return false;
        dist.push_back(v);
        prev_pos = pos + 1;
    } while (pos != std::string::npos);
    float total = 0.0f;
    for (float v : dist) total += v;
    for (float& v : dist) v /= total;
    return true;
}

// the history draw (samples/gpu/tbd.cpp:656-671)
static unsigned draw_history_age(tbd::CRand& rng, const std::vector<float>& dist)
{
    float cumulative = 0.0f;
    const float r = ((float)rng.rand()) / (float)tbd::CRand::kRandMax;
    for (unsigned i = 0; i < dist.size(); ++i) {
        cumulative += dist[i];
        if (r < cumulative) return i + 1;
    }
    return (unsigned)dist.size();
}

static void put_g(std::string& s, double v)  // ostream << double (precision 6, %g)
{
    char buf[64];
    std::snprintf(buf, sizeof buf, "%g", v);
    s += buf;
}

static void put_i(std::string& s, long long v)
{
    char buf[32];
    std::snprintf(buf, sizeof buf, "%lld", v);
    s += buf;
}

// App::writeTrackingOutputToFile (samples/gpu/tbd.cpp:946-1120).  frame_count
// = the sample's this->frame_id when it writes (frames processed).
bool write_tracking_output(const tbd::Tracker& tk, const std::vector<unsigned>& historyAges,
                                  tbd::TrajectoryMap& trajectoryMap, unsigned frame_count, const char* path,
                                  FILE* log, tbdk_scenario_metrics* out)
{
    std::string s;
    s += "history|";
    for (size_t i = 0; i < historyAges.size(); ++i) {
        if (i > 0) s += ",";
        put_i(s, historyAges[i]);
    }
    s += "\n";

    // idSwapsPerFrame(frame_id): sized so that no index can fall outside (the
    // reference writes out of bounds for a trajectory frame >= frame_id)
    size_t nsw = std::max<size_t>(frame_count, tk.truePositives.size());
    for (auto& kv : trajectoryMap)
        for (int fnum : kv.second.presentFrames)
            if (fnum >= 0) nsw = std::max(nsw, (size_t)fnum + 1);
    std::vector<int> idSwapsPerFrame(nsw, 0);
    std::map<int, int> numFragmentationsPerTrack;
    int numMostlyTracked = 0, numPartiallyTracked = 0, numMostlyLost = 0;
    for (auto& kv : trajectoryMap) {
        tbd::Trajectory& tr = kv.second;
        numFragmentationsPerTrack[tr.id] = 0;
        bool isNew = true, prevTracked = false;
        int prevTrackId = -1, numTrackedFrames = 0;
        for (size_t pfid = 0; pfid < tr.presentFrames.size(); ++pfid) {
            const int fnum = tr.presentFrames[pfid];
            const bool tracked = tr.isTrackedPerFrame[fnum];
            if (tracked) {
                const int trackId = tr.trackIdPerFrame[fnum];
                if (isNew) {
                    prevTrackId = trackId;
                } else if (trackId != prevTrackId) {
                    if (log)
                        std::fprintf(log, "[frame %d] target %d switched from track %d to track %d\n", fnum, tr.id,
                                     prevTrackId, trackId);
                    if (fnum >= 0) idSwapsPerFrame[(size_t)fnum]++;
                    prevTrackId = trackId;
                }
                numTrackedFrames++;
            }
            if (!isNew && !prevTracked && tracked) numFragmentationsPerTrack[tr.id]++;
            prevTracked = tracked;
            isNew = pfid == 0;  // the reference's lag: frames 0 and 1 both count as new
        }
        const double ratio = ((double)numTrackedFrames) / tr.presentFrames.size();
        if (ratio >= 0.8)
            numMostlyTracked++;
        else if (ratio > 0.2)
            numPartiallyTracked++;
        else
            numMostlyLost++;
    }

    for (auto& kv : trajectoryMap) {
        tbd::Trajectory& tr = kv.second;
        s += "object|";
        put_i(s, tr.id);
        s += "|";
        for (size_t pfid = 0; pfid < tr.presentFrames.size(); ++pfid) {
            if (pfid > 0) s += ";";
            const int fnum = tr.presentFrames[pfid];
            put_i(s, fnum);
            s += ",";
            put_i(s, tr.isTrackedPerFrame[fnum] ? 1 : 0);
            s += ",";
            put_i(s, tr.trackIdPerFrame[fnum]);
        }
        s += "|FM,";
        put_i(s, numFragmentationsPerTrack[tr.id]);
        s += "\n";
    }

    double totalBboxOverlap = 0.0;
    const size_t nf = tk.truePositives.size();
    for (size_t fnum = 0; fnum < nf; ++fnum) {
        s += "frame|";
        put_i(s, (long long)fnum);
        s += "|TP,";
        put_i(s, tk.truePositives[fnum]);
        s += ";FN,";
        put_i(s, tk.falseNegatives[fnum]);
        s += ";FP,";
        put_i(s, tk.falsePositives[fnum]);
        s += ";GT,";
        put_i(s, tk.groundTruths[fnum]);
        s += ";c,";
        put_i(s, tk.numMatches[fnum]);
        s += ";IDSW,";
        put_i(s, idSwapsPerFrame[fnum]);
        s += ";sum_di,";
        put_g(s, tk.bboxOverlap[fnum]);
        s += "\n";
        totalBboxOverlap += tk.bboxOverlap[fnum];
    }

    double motaNum = 0.0, amotaNum = 0.0, motaDen = 0.0, motpDen = 0.0;
    int64_t idsw = 0;
    for (size_t fnum = 0; fnum < nf; ++fnum) {
        motaNum += (tk.falseNegatives[fnum] + tk.falsePositives[fnum] + idSwapsPerFrame[fnum]);
        amotaNum += (tk.falseNegatives[fnum] + tk.falsePositives[fnum]);
        motaDen += tk.groundTruths[fnum];
        motpDen += tk.numMatches[fnum];
        idsw += idSwapsPerFrame[fnum];
    }
    const double mota = 1 - (motaNum / motaDen);
    const double amota = 1 - (amotaNum / motaDen);
    const double motp = totalBboxOverlap / motpDen;
    s += "scenario|MT,";
    put_i(s, numMostlyTracked);
    s += ";PT,";
    put_i(s, numPartiallyTracked);
    s += ";ML,";
    put_i(s, numMostlyLost);
    s += ";MOTA,";
    put_g(s, mota);
    s += ";A-MOTA,";
    put_g(s, amota);
    s += ";MOTP,";
    put_g(s, motp);
    s += "\n";

    if (out) {
        out->mt = numMostlyTracked;
        out->pt = numPartiallyTracked;
        out->ml = numMostlyLost;
        int fm = 0;
        for (auto& kv : numFragmentationsPerTrack) fm += kv.second;
        out->fm = fm;
        out->idsw = (int32_t)idsw;
        out->frames = (int32_t)nf;
        out->mota = mota;
        out->amota = amota;
        out->motp = motp;
    }
    if (path && path[0]) {
        FILE* f = std::fopen(path, "ab");  // ios::out | ios::app
        if (!f) return false;
        const bool ok = std::fwrite(s.data(), 1, s.size(), f) == s.size();
        return (std::fclose(f) == 0) && ok;
    }
    return true;
}

static tbd::TbdArgs to_args(const tbdk_tracker_args& a)
{
    tbd::TbdArgs t;
    t.costOfNonAssignment = a.cost_of_non_assignment;
    t.timeWindowSize = (unsigned)a.time_window_size;
    t.trackAgeThreshold = (unsigned)a.track_age_threshold;
    t.trackVisibilityThreshold = a.track_visibility_threshold;
    t.trackConfidenceThreshold = a.track_confidence_threshold;
    t.boundsXmin = a.bounds_xmin;
    t.boundsXmax = a.bounds_xmax;
    t.boundsYmin = a.bounds_ymin;
    t.boundsYmax = a.bounds_ymax;
    return t;
}

}  // namespace app
}  // namespace tbdk

// ---- C ABI ----
namespace tbdk {
namespace app {
void add_positions(tbd::TrajectoryMap& traj, const std::vector<tbd::Detection>& dets, int frame)
{
    // parseDetections' trajectory update (samples/gpu/tbd.cpp:1327-1338)
    for (const auto& d : dets) {
        if (d.id < 0) continue;
        auto it = traj.find(d.id);
        if (it == traj.end()) it = traj.emplace(d.id, tbd::Trajectory(d.id)).first;
        it->second.addPosition(frame, d.bbox);
    }
}
}  // namespace app
}  // namespace tbdk

using namespace tbdk;

extern "C" {

int tbdk_sequence_create(tbdk_sequence** out)
{
    if (!out) return TBDK_EINVAL;
    *out = new (std::nothrow) tbdk_sequence();
    return *out ? TBDK_OK : TBDK_ENOMEM;
}

int tbdk_sequence_destroy(tbdk_sequence* s)
{
    if (!s) return TBDK_EINVAL;
    delete s;
    return TBDK_OK;
}

int tbdk_sequence_parse_bbox_file(tbdk_sequence* s, int cls, const char* path, uint32_t num_frames)
{
    if (!s || !path || cls < 0 || cls > 1) return TBDK_EINVAL;
    s->error.clear();
    BboxTable& t = s->cls[cls];
    t.frames.clear();
    if (!app::parse_bbox_file(path, num_frames, t, s->poses, s->history, s->error)) return TBDK_EINVAL;
    return TBDK_OK;
}

const char* tbdk_sequence_error(const tbdk_sequence* s)
{
    return s ? s->error.c_str() : "";
}

int tbdk_sequence_info(const tbdk_sequence* s, int cls, int32_t* nframes, int32_t* nposes, int32_t* nhistory)
{
    if (!s || cls < 0 || cls > 1) return TBDK_EINVAL;
    if (nframes) *nframes = (int32_t)s->cls[cls].frames.size();
    if (nposes) *nposes = (int32_t)s->poses.size();
    if (nhistory) *nhistory = (int32_t)s->history.size();
    return TBDK_OK;
}

int tbdk_sequence_history(const tbdk_sequence* s, uint32_t* out, int cap, int* n)
{
    if (!s || !n || cap < 0 || (cap > 0 && !out)) return TBDK_EINVAL;
    for (int i = 0; i < cap && (size_t)i < s->history.size(); ++i) out[i] = s->history[(size_t)i];
    *n = (int)s->history.size();
    return TBDK_OK;
}

int tbdk_sequence_camera_pose(const tbdk_sequence* s, int index, double* out, int cap, int* n)
{
    if (!s || !n || index < 0 || cap < 0 || (cap > 0 && !out)) return TBDK_EINVAL;
    if ((size_t)index >= s->poses.size()) return TBDK_EINVAL;
    const auto& p = s->poses[(size_t)index];
    for (int i = 0; i < cap && (size_t)i < p.size(); ++i) out[i] = p[(size_t)i];
    *n = (int)p.size();
    return TBDK_OK;
}

int tbdk_sequence_detections(const tbdk_sequence* s, int cls, int frame, tbdk_trajectories* traj,
                             tbdk_detection* out, int cap, int* n)
{
    if (!s || !n || cls < 0 || cls > 1 || cap < 0 || (cap > 0 && !out)) return TBDK_EINVAL;
    std::vector<tbd::Detection> dets;
    app::parse_detections(s->cls[cls], frame, dets, traj ? &traj->map : nullptr);
    for (int i = 0; i < cap && (size_t)i < dets.size(); ++i) {
        const tbd::Detection& d = dets[(size_t)i];
        out[i].id = d.id;
        out[i].x = d.bbox.x;
        out[i].y = d.bbox.y;
        out[i].width = d.bbox.width;
        out[i].height = d.bbox.height;
        out[i].confidence = d.confidence;
    }
    *n = (int)dets.size();
    return TBDK_OK;
}

int tbdk_trajectories_create(tbdk_trajectories** out)
{
    if (!out) return TBDK_EINVAL;
    *out = new (std::nothrow) tbdk_trajectories();
    return *out ? TBDK_OK : TBDK_ENOMEM;
}

int tbdk_trajectories_destroy(tbdk_trajectories* t)
{
    if (!t) return TBDK_EINVAL;
    delete t;
    return TBDK_OK;
}

int tbdk_trajectories_add_position(tbdk_trajectories* t, int id, int frame, int x, int y, int w, int h)
{
    if (!t || id < 0) return TBDK_EINVAL;
    auto it = t->map.find(id);
    if (it == t->map.end()) it = t->map.emplace(id, tbd::Trajectory(id)).first;
    it->second.addPosition(frame, Rect(x, y, w, h));
    return TBDK_OK;
}

int tbdk_trajectories_count(const tbdk_trajectories* t, int* n)
{
    if (!t || !n) return TBDK_EINVAL;
    *n = (int)t->map.size();
    return TBDK_OK;
}

int tbdk_rand_create(uint32_t seed, tbdk_rand** out)
{
    if (!out) return TBDK_EINVAL;
    *out = new (std::nothrow) tbdk_rand(seed);
    return *out ? TBDK_OK : TBDK_ENOMEM;
}

int tbdk_rand_destroy(tbdk_rand* r)
{
    if (!r) return TBDK_EINVAL;
    delete r;
    return TBDK_OK;
}

int tbdk_rand_next(tbdk_rand* r, int32_t* out)
{
    if (!r || !out) return TBDK_EINVAL;
    *out = r->r.rand();
    return TBDK_OK;
}

int tbdk_history_age(tbdk_rand* r, const float* dist, int n, uint32_t* age)
{
    if (!r || !dist || n <= 0 || !age) return TBDK_EINVAL;
    *age = app::draw_history_age(r->r, std::vector<float>(dist, dist + n));
    return TBDK_OK;
}

int tbdk_parse_history_distribution(const char* s, float* out, int cap, int* n)
{
    if (!s || !n || cap < 0 || (cap > 0 && !out)) return TBDK_EINVAL;
    std::vector<float> d;
    if (!app::parse_history_distribution(s, d)) return TBDK_EINVAL;
    for (int i = 0; i < cap && (size_t)i < d.size(); ++i) out[i] = d[(size_t)i];
    *n = (int)d.size();
    return TBDK_OK;
}

int tbdk_tracker_set_rand(tbdk_tracker* t, tbdk_rand* r)
{
    if (!t) return TBDK_EINVAL;
    t->tracker.setRand(r ? &r->r : nullptr);
    return TBDK_OK;
}

int tbdk_tracker_step_traj(tbdk_tracker* t, const tbdk_detection* dets, int ndets, int frame_id,
                           const tbdk_prediction* preds, int npreds, tbdk_trajectories* traj, tbdk_frame_metrics* m)
{
    if (!t || ndets < 0 || (ndets > 0 && !dets) || npreds < 0 || (npreds > 0 && !preds)) return TBDK_EINVAL;
    t->dets.resize((size_t)ndets);
    for (int i = 0; i < ndets; ++i) {
        tbd::Detection& d = t->dets[(size_t)i];
        d.id = dets[i].id;
        d.frame_id = frame_id;
        d.bbox = Rect(dets[i].x, dets[i].y, dets[i].width, dets[i].height);
        d.confidence = dets[i].confidence;
    }
    t->preds.resize((size_t)npreds);
    for (int i = 0; i < npreds; ++i)
        t->preds[(size_t)i] = tbd::Prediction{preds[i].track_id, preds[i].valid, preds[i].cx, preds[i].cy};
    t->tracker.performTrackingStep(t->dets, frame_id, t->preds.data(), npreds, traj ? &traj->map : nullptr);
    if (m) {
        std::memset(m, 0, sizeof(*m));
        const tbd::Tracker& k = t->tracker;
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

int tbdk_tracker_reset(tbdk_tracker* t)
{
    if (!t) return TBDK_EINVAL;
    t->tracker.reset();
    return TBDK_OK;
}

int tbdk_track_buffer_create(int nslots, tbdk_track_buffer** out)
{
    if (!out || nslots <= 0) return TBDK_EINVAL;
    *out = new (std::nothrow) tbdk_track_buffer();
    if (!*out) return TBDK_ENOMEM;
    (*out)->slots.resize((size_t)nslots);
    return TBDK_OK;
}

int tbdk_track_buffer_destroy(tbdk_track_buffer* b)
{
    if (!b) return TBDK_EINVAL;
    delete b;
    return TBDK_OK;
}

int tbdk_tracker_store_tracks(tbdk_tracker* t, tbdk_track_buffer* b, int slot)
{
    if (!t || !b || slot < 0 || (size_t)slot >= b->slots.size()) return TBDK_EINVAL;
    b->slots[(size_t)slot] = t->tracker.getTracks();
    return TBDK_OK;
}

int tbdk_tracker_load_tracks(tbdk_tracker* t, const tbdk_track_buffer* b, int slot)
{
    if (!t) return TBDK_EINVAL;
    if (slot < 0) {  // setTracks(empty)
        t->tracker.setTracks({});
        return TBDK_OK;
    }
    if (!b || (size_t)slot >= b->slots.size()) return TBDK_EINVAL;
    t->tracker.setTracks(b->slots[(size_t)slot]);
    return TBDK_OK;
}

int tbdk_tracking_write(const tbdk_tracker* t, const uint32_t* history_ages, int nages, int frame_count,
                        tbdk_trajectories* traj, const char* path, int log_switches, tbdk_scenario_metrics* out)
{
    if (!t || !traj || nages < 0 || (nages > 0 && !history_ages) || frame_count < 0) return TBDK_EINVAL;
    std::vector<unsigned> ages(history_ages, history_ages + nages);
    return app::write_tracking_output(t->tracker, ages, traj->map, (unsigned)frame_count, path,
                                      log_switches ? stdout : nullptr, out)
               ? TBDK_OK
               : TBDK_EINVAL;
}

int tbdk_app_default_args(tbdk_app_args* a)
{
    if (!a) return TBDK_EINVAL;
    std::memset(a, 0, sizeof(*a));
    tbdk_tracker_default_args(&a->tracker);
    a->num_tracking_iters = 1;      // samples/gpu/tbd.cpp:256-257
    a->num_tracking_frames = 100;
    a->rand_seed = 1;               // rand() never seeded
    return TBDK_OK;
}

// App::run, tracking section (samples/gpu/tbd.cpp:479-706, 823-841) with
// ground-truth / external detections from the bbox files.
int tbdk_app_run(const tbdk_app_args* a, tbdk_app_result* res)
{
    if (!a || a->num_tracking_frames < 0 || a->num_tracking_iters < 0) return TBDK_EINVAL;
    const char* files[2] = {a->pedestrian_bbox_filename, a->vehicle_bbox_filename};
    const char* outs[2] = {a->pedestrian_tracking_filepath, a->vehicle_tracking_filepath};
    const bool track[2] = {files[0] && files[0][0], files[1] && files[1][0]};
    if (!track[0] && !track[1]) return TBDK_EINVAL;  // the sample would run its HOG detector instead
    if (res) std::memset(res, 0, sizeof(*res));

    std::vector<float> dist(1, 1.0f);
    if (a->history_distribution && a->history_distribution[0] &&
        !app::parse_history_distribution(a->history_distribution, dist))
        return TBDK_EINVAL;

    tbdk_sequence seq;
    for (int c = 0; c < 2; ++c) {
        if (!track[c]) continue;
        if (!app::parse_bbox_file(files[c], (unsigned)a->num_tracking_frames, seq.cls[c], seq.poses, seq.history,
                                  seq.error)) {
            if (a->verbose) std::fprintf(stdout, "error: %s\n", seq.error.c_str());
            return TBDK_EINVAL;
        }
    }
    const bool use_provided = !seq.history.empty();
    if (use_provided && seq.history.size() < (size_t)a->num_tracking_frames) return TBDK_EINVAL;

    tbd::CRand rng(a->rand_seed);
    const tbd::TbdArgs targs = app::to_args(a->tracker);
    const size_t H = dist.size();
    for (int iter = 0; iter < a->num_tracking_iters; ++iter) {
        tbd::TrajectoryMap traj[2];
        std::vector<std::vector<tbd::Track>> buf[2];
        for (int c = 0; c < 2; ++c) buf[c].assign(H, {});
        std::vector<unsigned> historyAges;
        tbd::Tracker trackers[2] = {tbd::Tracker(targs), tbd::Tracker(targs)};
        for (int c = 0; c < 2; ++c) trackers[c].setRand(&rng);
        std::vector<tbd::Detection> dets[2];
        std::vector<tbd::Track> prior;
        unsigned frame_id = 0;
        for (; frame_id < (unsigned)a->num_tracking_frames; ++frame_id) {
            for (int c = 0; c < 2; ++c) app::parse_detections(seq.cls[c], (int)frame_id, dets[c], &traj[c]);
            if (frame_id == 0) {
                for (int c = 0; c < 2; ++c) {
                    for (auto& v : buf[c]) v.clear();
                    trackers[c].reset();
                }
            }
            const unsigned age = use_provided ? seq.history[frame_id] : app::draw_history_age(rng, dist);
            historyAges.push_back(age);
            for (int c = 0; c < 2; ++c) {
                prior.clear();
                if (frame_id >= age) prior = buf[c][(frame_id - age) % H];
                trackers[c].setTracks(prior);
            }
            for (int c = 0; c < 2; ++c)
                if (track[c]) trackers[c].performTrackingStep(dets[c], (int)frame_id, nullptr, 0, &traj[c]);
            for (int c = 0; c < 2; ++c) buf[c][frame_id % H] = trackers[c].getTracks();
            if (res) {
                res->frames++;
                res->detections += (int64_t)(dets[0].size() + dets[1].size());
            }
        }
        if (a->write_tracking) {
            for (int c = 0; c < 2; ++c) {
                if (!outs[c] || !outs[c][0]) continue;
                tbdk_scenario_metrics m;
                if (!app::write_tracking_output(trackers[c], historyAges, traj[c], frame_id, outs[c],
                                                a->verbose ? stdout : nullptr, &m))
                    return TBDK_EINVAL;
                if (res) res->scenario[c] = m;
            }
        } else if (res) {
            for (int c = 0; c < 2; ++c)
                app::write_tracking_output(trackers[c], historyAges, traj[c], frame_id, nullptr, nullptr,
                                           &res->scenario[c]);
        }
    }
    return TBDK_OK;
}

}  // extern "C"
