// tracker_solver_check.cpp — the tracker's first-round assignment on value
// kinds (the default) against the same tracker solving every round on the
// dense cost matrix (Tracker::setDenseSolver), frame by frame: assignments,
// every track field and the per-frame metrics must be identical.  Scenarios:
// duplicated and clustered boxes (ties, several zeros per row and column,
// step-3/step-4 rounds), dropouts (padding columns), clutter (padding rows),
// zero-size boxes (0/0 costs), touching boxes and padding values below 1,
// at 1 and outside (0, 1e7) (the dense path), frames without detections.
// Build: g++ -std=c++17 -I opencv_amd/csrc tests/cpp/tracker_solver_check.cpp opencv_amd/csrc/tbd_tracker.cpp
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "tbd_tracker.hpp"

using namespace tbdk::tbd;

static bool same(double a, double b) { return (std::isnan(a) && std::isnan(b)) || std::memcmp(&a, &b, 8) == 0; }

static int fail(int scen, int f, const char* what)
{
    printf("MISMATCH scenario %d frame %d: %s\n", scen, f, what);
    return 1;
}

int main()
{
    const double pads[] = {10.0, 0.3, 0.5, 1.0, 0.0, -1.0, 1e8, 20.0};
    long frames = 0, multi = 0;
    for (int scen = 0; scen < 64; ++scen) {
        std::mt19937 rng(1234u + (unsigned)scen);
        auto U = [&](int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(rng); };
        auto P = [&]() { return std::uniform_real_distribution<double>(0.0, 1.0)(rng); };
        TbdArgs a;
        a.costOfNonAssignment = pads[scen % 8];
        if (scen % 3 == 1) { a.boundsXmin = 0; a.boundsXmax = 640; a.boundsYmin = 0; a.boundsYmax = 480; }
        a.trackAgeThreshold = (unsigned)U(2, 10);
        Tracker fast(a), dense(a);
        dense.setDenseSolver(true);
        const int W = 640, H = 480;
        const int nobj = U(1, 90);
        const double cluster = (scen / 8) % 2 ? 0.0 : 0.6;  // share of objects on a few spots
        std::vector<double> x(nobj), y(nobj), vx(nobj), vy(nobj);
        std::vector<int> w(nobj), h(nobj);
        for (int o = 0; o < nobj; ++o) {
            if (P() < cluster) {
                x[o] = 100 + 50 * U(0, 2);
                y[o] = 100 + 40 * U(0, 2);
                w[o] = 40 + 10 * U(0, 1);
                h[o] = 40;
                vx[o] = vy[o] = U(0, 1);
            } else {
                x[o] = U(0, W - 40);
                y[o] = U(0, H - 40);
                w[o] = U(scen % 5 == 0 ? 0 : 4, 120);
                h[o] = U(scen % 5 == 0 ? 0 : 4, 120);
                vx[o] = U(-5, 5);
                vy[o] = U(-5, 5);
            }
        }
        const double dropout = 0.05 * (scen % 4), clutter = 0.1 * (scen % 7);
        for (int f = 0; f < 60; ++f) {
            std::vector<Detection> dets;
            for (int o = 0; o < nobj; ++o) {
                x[o] += vx[o];
                y[o] += vy[o];
                if (x[o] < -30 || x[o] > W - 10) vx[o] = -vx[o];
                if (y[o] < -30 || y[o] > H - 10) vy[o] = -vy[o];
                if (P() < dropout) continue;
                Detection d;
                d.id = o;
                d.frame_id = f;
                const int j = scen % 2 ? U(-2, 2) : 0;
                d.bbox = Rect((int)x[o] + j, (int)y[o] + j, std::max(0, w[o] + j), std::max(0, h[o] - j));
                d.confidence = P() < 0.1 ? 0.2 * P() : 1.0;
                dets.push_back(d);
                if (P() < 0.05) dets.push_back(d);  // a duplicated detection
            }
            const int extra = (int)std::floor(clutter * nobj * P());
            for (int k = 0; k < extra; ++k) {
                Detection d;
                d.id = -1;
                d.frame_id = f;
                d.bbox = Rect(U(-20, W), U(-20, H), U(0, 80), U(0, 80));
                dets.push_back(d);
            }
            if (scen % 4 == 3 && f % 7 == 6) dets.clear();  // a frame without detections (padding columns only)
            std::vector<Detection> d2 = dets;
            fast.performTrackingStep(dets, f);
            dense.performTrackingStep(d2, f);
            frames++;
            const auto& A = fast.getTracks();
            const auto& B = dense.getTracks();
            if (fast.lastAssignments != dense.lastAssignments) return fail(scen, f, "assignments");
            if (fast.createdIds != dense.createdIds || fast.deletedIds != dense.deletedIds) return fail(scen, f, "ids");
            if (A.size() != B.size()) return fail(scen, f, "track count");
            for (size_t i = 0; i < A.size(); ++i) {
                const Track &p = A[i], &q = B[i];
                const Rect &bp = p.bboxes.back(), &bq = q.bboxes.back();
                if (p.id != q.id || bp.x != bq.x || bp.y != bq.y || bp.width != bq.width || bp.height != bq.height ||
                    p.predPosition.x != q.predPosition.x || p.predPosition.y != q.predPosition.y ||
                    p.age != q.age || p.totalVisibleCount != q.totalVisibleCount ||
                    !same(p.maxConfidence, q.maxConfidence) || !same(p.avgConfidence, q.avgConfidence) ||
                    !same(p.bboxOverlap, q.bboxOverlap))
                    return fail(scen, f, "track fields");
            }
            if (fast.truePositives != dense.truePositives || fast.falseNegatives != dense.falseNegatives ||
                fast.falsePositives != dense.falsePositives || fast.numMatches != dense.numMatches)
                return fail(scen, f, "metrics");
            if (!same(fast.bboxOverlap.back(), dense.bboxOverlap.back())) return fail(scen, f, "overlap sum");
            multi += fast.lastRounds > 1;
        }
    }
    printf("tracker solver ok: %ld frames, %ld with more than one round\n", frames, multi);
    return multi > 0 ? 0 : 2;  // the scenarios must reach the dense rounds
}
