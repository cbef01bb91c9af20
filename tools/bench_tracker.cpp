// bench_tracker.cpp — host-only timing of the native tracker step on the
// bench workload's ground-truth detections (1080p x 128 synthetic objects).
// Build: g++ -O3 -std=c++17 -I opencv_amd/csrc tools/bench_tracker.cpp opencv_amd/csrc/tbd_tracker.cpp
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "synth_spec.h"
#include "tbd_tracker.hpp"

using namespace tbdk::tbd;

int main(int argc, char** argv)
{
    const int W = 1920, H = 1080, nobj = argc > 1 ? atoi(argv[1]) : 128, nframes = 300;
    const bool frame_bounds = argc > 2 && argv[2][0] == 'f';
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    std::vector<syn_object> objs(nobj);
    syn_make_objects(20261015u, W, H, nobj, objs.data());
    // the detections of every frame first, so the timed loop runs only the tracker
    std::vector<std::vector<Detection>> seq(nframes);
    for (int f = 0; f < nframes; ++f)
        for (int o = 0; o < nobj; ++o) {
            syn_pose p;
            syn_pose_at(&objs[o], W, H, f, &p);
            int32_t b[4];
            if (!syn_gt_box(&p, W, H, b)) continue;
            Detection d;
            d.id = o; d.frame_id = f; d.bbox = Rect(b[0], b[1], b[2], b[3]); d.confidence = 1.0;
            seq[f].push_back(d);
        }
    TbdArgs a;
    if (frame_bounds) { a.boundsXmax = W; a.boundsYmax = H; }
    double best = 1e30;
    uint64_t chk = 0;
    long sum_tracks = 0;
    for (int rep = 0; rep < reps; ++rep) {  // the best of `reps` passes over the sequence
        Tracker tr(a);
        double tot = 0;
        chk = 0;
        sum_tracks = 0;
        for (int f = 0; f < nframes; ++f) {
            std::vector<Detection> dets = seq[f];
            auto t0 = std::chrono::steady_clock::now();
            tr.performTrackingStep(dets, f);
            auto t1 = std::chrono::steady_clock::now();
            if (f >= 20) tot += std::chrono::duration<double, std::micro>(t1 - t0).count();
            sum_tracks += (long)tr.getTracks().size();
            for (auto& t : tr.getTracks()) {
                const Rect& b = t.bboxes.back();
                const Rect& p = t.predPosition;
                for (long v : {(long)t.id, (long)b.x, (long)b.y, (long)b.width, (long)b.height, (long)p.x, (long)p.y,
                               (long)t.age, (long)t.totalVisibleCount, (long)(t.maxConfidence * 1e6),
                               (long)(t.bboxOverlap * 1e9)})
                    chk = chk * 1000003u + (uint64_t)v;
            }
            chk = chk * 7u + (uint64_t)tr.truePositives.back();
        }
        best = std::min(best, tot / (nframes - 20));
    }
    printf("tracker step: %.1f us/frame (best of %d), mean tracks %.1f, checksum %016llx\n", best, reps,
           (double)sum_tracks / nframes, (unsigned long long)chk);
    return 0;
}
