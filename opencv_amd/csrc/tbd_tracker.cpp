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

// the zero test of the reduced cost (equalsZero, tbd.hpp:178-181) on an entry
// stored as `value - colMin` (step 2's subtraction, :563-578)
static inline bool zero_after(double value, double colMin)
{
    const double v = value - colMin;
    return std::fabs(v) < 0.00000001;
}

// zero bits of one row's default entries: bit c = zero_after(a, colMin[c])
TBDK_SOLVER_CLONES static void zero_bits_uniform(double a, const double* __restrict colMin, unsigned n,
                                                 uint64_t* __restrict bits)
{
    for (unsigned w = 0; w * 64 < n; ++w) {
        const unsigned c0 = w * 64, c1 = std::min(n, c0 + 64);
        uint64_t m = 0;
        for (unsigned c = c0; c < c1; ++c) m |= (uint64_t)(std::fabs(a - colMin[c]) < 0.00000001) << (c - c0);
        bits[w] = m;
    }
}

// first index of sorted a[0..n) whose value is >= key (std::lower_bound), with
// conditional moves instead of branches
static inline unsigned lower_bound_cmov(const int* a, unsigned n, long key)
{
    const int* base = a;
    while (n > 1) {
        const unsigned half = n / 2;
        base = ((long)base[half - 1] < key) ? base + half : base;
        n -= half;
    }
    return (unsigned)(base - a) + (unsigned)(n == 1 && (long)*base < key);
}

static inline void set_bit(uint64_t* bits, unsigned c, bool v)
{
    const uint64_t b = (uint64_t)1 << (c & 63);
    bits[c >> 6] = v ? (bits[c >> 6] | b) : (bits[c >> 6] & ~b);
}

// calculateCostMatrix + solveAssignmentProblem + classifyAssignments
// (tbd.cpp:333-891) on a flat n x n matrix.  The reference's operation order
// on every matrix entry is kept (row minima, column minima, the step-4
// subtract/add of mu), so every comparison sees the same doubles; only the
// loop nests are reorganised for the cache and the vector units: column
// minima are accumulated row by row (same r order per column), the zero
// pattern and its row/column counts are rebuilt in one pass, and the
// "row assigned to column c" lookup of the cover step is an inverse map.
//
// The first round does not build the matrix.  A track row holds three kinds of
// entries: the detections its predicted box overlaps (a handful, found by an
// x-sorted sweep), 1.0 for every other detection (computeBoundingBoxOverlap
// returns exactly 0.0 for disjoint boxes) and the padding; a padding row is
// padding throughout.  After step 1 every entry of a kind is the same double
// (`1.0 - m`, `pad - m`), so each column's minimum is the smallest such value
// among the rows without an overlap in that column, or an overlap entry, and
// an entry's zero test is `fabs(value - colMin[c]) < 1e-8` on the same two
// doubles the dense pass subtracts.  The zero pattern is kept as one bit per
// entry, the step-2 assignment (:585-714) scans bits.  Only when that round
// leaves rows unassigned (about 2 % of the bench's frames) is the matrix built,
// entry by entry with the same operations, and the dense rounds continue with
// step 3.  Minima use the reference's `(v < m) ? v : m` step, whose result does
// not depend on the order of the values when no -0.0 can occur (a padding
// value that is not in (0, huge) takes the dense path).
void Tracker::solveAssignment(std::vector<Detection>& dets, std::vector<int>& assignments,
                              std::vector<unsigned>& unassignedTracks, std::vector<unsigned>& unassignedDetections)
{
    const unsigned nT = (unsigned)tracks.size(), nD = (unsigned)dets.size();
    const unsigned n = std::max(nT, nD);
    const double huge = 10000000.0;
    const double pad = args.costOfNonAssignment * 2;
    detKey.resize(nD);
    detOrder.resize(nD);
    int maxW = 0;
    for (unsigned j = 0; j < nD; ++j) {  // (x0, index) packed in one ordered key
        detKey[j] = ((uint64_t)((uint32_t)dets[j].bbox.x ^ 0x80000000u) << 32) | j;
        maxW = std::max(maxW, dets[j].bbox.width);
    }
    // detections by left edge: a track row only visits the detections whose x-range
    // can touch its box; all others are strictly separated, where the reference's
    // computeBoundingBoxOverlap returns exactly 0.0 (cost exactly 1.0)
    std::sort(detKey.begin(), detKey.end());
    for (unsigned k = 0; k < nD; ++k) detOrder[k] = (unsigned)detKey[k];
    sortedX0.resize(nD); sortedX1.resize(nD); sortedY0.resize(nD); sortedY1.resize(nD); sortedArea.resize(nD);
    for (unsigned k = 0; k < nD; ++k) {
        const Rect& b = dets[detOrder[k]].bbox;
        sortedX0[k] = b.x; sortedX1[k] = b.x + b.width; sortedY0[k] = b.y; sortedY1[k] = b.y + b.height;
        sortedArea[k] = b.area();
    }
    assignmentPerRow.assign(n, n);
    if (n == 0) return;
    // calculateCostMatrix (:333-351): the overlap entries of every track row
    exStart.resize(nT + 1);
    exCol.clear();
    exVal.clear();
    cand.resize(nD);
    for (unsigned r = 0; r < nT; ++r) {
        exStart[r] = (unsigned)exCol.size();
        const Rect& p = tracks[r].predPosition;
        const int px0 = p.x, py0 = p.y, px1 = p.x + p.width, py1 = p.y + p.height, pa = p.area();
        const unsigned lb = lower_bound_cmov(sortedX0.data(), nD, (long)px0 - maxW);
        const unsigned ub = lower_bound_cmov(sortedX0.data(), nD, (long)px1 + 1);  // the first x0 > px1
        // boxes that touch or overlap (computeBoundingBoxOverlap's xright >= xleft and
        // ybottom >= ytop, :1094-1097), gathered without branches
        unsigned nc = 0;
        for (unsigned k = lb; k < ub; ++k) {
            cand[nc] = k;
            nc += (unsigned)((sortedX1[k] >= px0) & (sortedY0[k] <= py1) & (sortedY1[k] >= py0));
        }
        for (unsigned i = 0; i < nc; ++i) {
            const unsigned k = cand[i];
            const int xl = std::max(px0, sortedX0[k]), xr = std::min(px1, sortedX1[k]);
            const int yt = std::max(py0, sortedY0[k]), yb = std::min(py1, sortedY1[k]);
            const double inter = (double)(xr - xl) * (double)(yb - yt);
            const double uni = (double)(pa + sortedArea[k]) - inter;
            exCol.push_back(detOrder[k]);
            exVal.push_back(1.0 - inter / uni);
        }
    }
    exStart[nT] = (unsigned)exCol.size();

    rowZeros.resize(n);
    colZeros.resize(n);
    colLast.resize(n);
    colRow.resize(n);
    rowA.assign(n, 0);
    colA.assign(n, 0);
    rowM.resize(n);
    colM.resize(n);
    colRow.assign(n, n);
    unsigned numAssigned = 0;
    lastRounds = 1;
    auto assign = [&](unsigned r, unsigned c) {
        rowA[r] = colA[c] = 1;
        assignmentPerRow[r] = c;
        colRow[c] = r;
        numAssigned++;
    };

    const bool sparse = !denseSolver && pad > 0.0 && pad < huge;
    bool dense_zero_pass = true;  // the dense loop starts with step 2's zero pattern
    if (sparse) {
        // step 1 (:494-516): every row's minimum over its value kinds
        rowMinV.resize(nT);
        rowDef.resize(nT);
        rowPadV.resize(nT);
        exValR.resize(exVal.size());
        for (unsigned r = 0; r < nT; ++r) {
            double m = huge;
            if (exStart[r + 1] - exStart[r] < nD) m = (1.0 < m) ? 1.0 : m;
            for (unsigned k = exStart[r]; k < exStart[r + 1]; ++k) m = (exVal[k] < m) ? exVal[k] : m;
            if (n > nD) m = (pad < m) ? pad : m;
            rowMinV[r] = m;
            rowDef[r] = 1.0 - m;
            rowPadV[r] = pad - m;
            for (unsigned k = exStart[r]; k < exStart[r + 1]; ++k) exValR[k] = exVal[k] - m;
        }
        const double padRowV = pad - ((pad < huge) ? pad : huge);  // rows nT..n-1
        // step 2's column minima (:539-561)
        colExStart.assign(nD + 1, 0);
        for (unsigned k = 0; k < exCol.size(); ++k) colExStart[exCol[k] + 1]++;
        for (unsigned c = 0; c < nD; ++c) colExStart[c + 1] += colExStart[c];
        colExRow.resize(exCol.size());
        colExVal.resize(exCol.size());
        colFill.assign(colExStart.begin(), colExStart.end() - 1);
        for (unsigned r = 0; r < nT; ++r)
            for (unsigned k = exStart[r]; k < exStart[r + 1]; ++k) {
                const unsigned at = colFill[exCol[k]]++;
                colExRow[at] = r;
                colExVal[at] = exValR[k];
            }
        defOrder.resize(nT);
        for (unsigned r = 0; r < nT; ++r) defOrder[r] = r;
        if (!(nT < n && padRowV == 0.0))
            std::sort(defOrder.begin(), defOrder.end(), [&](unsigned a, unsigned b) { return rowDef[a] < rowDef[b]; });
        colMin.assign(n, huge);
        // with padding rows (value pad - pad = +0.0) and every other entry >= +0.0
        // (v - m with m the row's minimum), every column's minimum is +0.0
        const bool zeroMins = nT < n && padRowV == 0.0;
        if (zeroMins) std::fill(colMin.begin(), colMin.begin() + nD, 0.0);
        for (unsigned c = 0; !zeroMins && c < nD; ++c) {
            double cm = huge;
            const unsigned e0 = colExStart[c], e1 = colExStart[c + 1];
            for (unsigned r : defOrder) {  // the smallest 1.0 - m of the rows with a 1.0 entry here
                bool ex = false;
                for (unsigned k = e0; k < e1; ++k) ex |= colExRow[k] == r;
                if (!ex) {
                    cm = (rowDef[r] < cm) ? rowDef[r] : cm;
                    break;
                }
            }
            for (unsigned k = e0; k < e1; ++k) cm = (colExVal[k] < cm) ? colExVal[k] : cm;
            if (nT < n) cm = (padRowV < cm) ? padRowV : cm;
            colMin[c] = cm;
        }
        double cmPad = huge;  // columns nD..n-1 (track rows only: nT == n)
        if (n > nD)
            for (unsigned r = 0; r < nT; ++r) cmPad = (rowPadV[r] < cmPad) ? rowPadV[r] : cmPad;
        for (unsigned c = nD; c < n; ++c) colMin[c] = cmPad;
        double cmLo = huge, cmHi = -huge;
        for (unsigned c = 0; c < nD; ++c) {
            cmLo = std::min(cmLo, colMin[c]);
            cmHi = std::max(cmHi, colMin[c]);
        }
        // the zero pattern after the column minima, one bit per entry
        const unsigned W = (n + 63) / 64;
        zbits.assign((size_t)n * W, 0);
        if (nT < n) {  // padding rows: one pattern
            zero_bits_uniform(padRowV, colMin.data(), n, &zbits[(size_t)nT * W]);
            for (unsigned r = nT + 1; r < n; ++r)
                std::memcpy(&zbits[(size_t)r * W], &zbits[(size_t)nT * W], W * sizeof(uint64_t));
        }
        for (unsigned r = 0; r < nT; ++r) {
            uint64_t* b = &zbits[(size_t)r * W];
            const double a = rowDef[r];
            // no 1.0 entry can be a zero when a is 1e-8 or more away from every column minimum
            if (nD && !(a - cmHi >= 0.00000001) && !(a - cmLo <= -0.00000001))
                zero_bits_uniform(a, colMin.data(), nD, b);
            for (unsigned k = exStart[r]; k < exStart[r + 1]; ++k)
                set_bit(b, exCol[k], zero_after(exValR[k], colMin[exCol[k]]));
            if (n > nD && zero_after(rowPadV[r], cmPad))
                for (unsigned c = nD; c < n; ++c) set_bit(b, c, true);
        }
        std::fill(colZeros.begin(), colZeros.end(), 0u);
        for (unsigned r = 0; r < std::min(n, nT + 1); ++r) {  // track rows, then the first padding row
            const uint64_t* b = &zbits[(size_t)r * W];
            const unsigned reps = r < nT ? 1 : n - nT, last = r < nT ? r : n - 1;
            unsigned cnt = 0;
            for (unsigned w = 0; w < W; ++w)
                for (uint64_t m = b[w]; m; m &= m - 1) {
                    const unsigned c = w * 64 + (unsigned)__builtin_ctzll(m);
                    colZeros[c] += reps;
                    colLast[c] = last;
                    cnt++;
                }
            rowZeros[r] = cnt;
        }
        for (unsigned r = nT + 1; r < n; ++r) rowZeros[r] = rowZeros[nT];
        // step 2's assignment (:585-714) on the bits
        colAbits.assign(W, 0);
        auto assign_b = [&](unsigned r, unsigned c) {
            assign(r, c);
            colAbits[c >> 6] |= (uint64_t)1 << (c & 63);
        };
        bool made = true;
        while (made) {
            made = false;
            for (unsigned r = 0; r < n; ++r) {  // rows with exactly one zero (:607-636)
                if (rowA[r] || rowZeros[r] != 1) continue;
                const uint64_t* b = &zbits[(size_t)r * W];
                unsigned w = 0;
                while (!b[w]) ++w;
                const unsigned c = w * 64 + (unsigned)__builtin_ctzll(b[w]);
                if (!colA[c]) {
                    assign_b(r, c);
                    made = true;
                }
            }
            for (unsigned c = 0; c < n; ++c) {  // columns with exactly one zero (:639-668)
                if (colA[c] || colZeros[c] != 1) continue;
                const unsigned r = colLast[c];
                if (!rowA[r]) {
                    assign_b(r, c);
                    made = true;
                }
            }
            if (!made) {  // first free zero of every unassigned row (:672-714)
                for (unsigned r = 0; r < n; ++r) {
                    if (rowA[r]) continue;
                    const uint64_t* b = &zbits[(size_t)r * W];
                    for (unsigned w = 0; w < W; ++w) {
                        const uint64_t m = b[w] & ~colAbits[w];
                        if (m) {
                            assign_b(r, w * 64 + (unsigned)__builtin_ctzll(m));
                            made = true;
                            break;
                        }
                    }
                }
            }
        }
        if (numAssigned < n) {
            // the dense rounds continue from step 3: the matrix and zero pattern as
            // the dense first round leaves them (each entry `(raw - m) - colMin[c]`)
            cost.resize((size_t)n * n);
            zero.resize((size_t)n * n);
            for (unsigned r = 0; r < n; ++r) {
                double* row = &cost[(size_t)r * n];
                if (r < nT) {
                    for (unsigned c = 0; c < nD; ++c) row[c] = rowDef[r];
                    for (unsigned k = exStart[r]; k < exStart[r + 1]; ++k) row[exCol[k]] = exValR[k];
                    for (unsigned c = nD; c < n; ++c) row[c] = rowPadV[r];
                } else {
                    for (unsigned c = 0; c < n; ++c) row[c] = padRowV;
                }
                const uint64_t* b = &zbits[(size_t)r * W];
                for (unsigned c = 0; c < n; ++c) {
                    row[c] -= colMin[c];
                    zero[(size_t)r * n + c] = (uint8_t)((b[c >> 6] >> (c & 63)) & 1);
                }
            }
            dense_zero_pass = false;
        }
    } else {
        // the dense first round: calculateCostMatrix fused with step 1, the row
        // minima (:494-516), and step 2's column minima
        cost.resize((size_t)n * n);
        zero.resize((size_t)n * n);
        colMin.assign(n, huge);
        for (unsigned r = 0; r < n; ++r) {
            double* row = &cost[(size_t)r * n];
            unsigned c0 = 0;
            if (r < nT) {
                for (unsigned j = 0; j < nD; ++j) row[j] = 1.0;
                for (unsigned k = exStart[r]; k < exStart[r + 1]; ++k) row[exCol[k]] = exVal[k];
                c0 = nD;
            }
            for (unsigned c = c0; c < n; ++c) row[c] = pad;
            sub_row_min_and_colmin(row, n, row_min(row, n, huge), colMin.data());
        }
    }
    if (numAssigned < n) {
        // the column minima's subtraction is fused into the dense first round's zero pass
        bool first = dense_zero_pass;
        while (true) {  // (:585-887)
            if (dense_zero_pass) {
                std::fill(colZeros.begin(), colZeros.end(), 0u);
                for (unsigned r = 0; r < n; ++r)
                    rowZeros[r] = zero_row(&cost[(size_t)r * n], first ? colMin.data() : nullptr, n,
                                           &zero[(size_t)r * n], colZeros.data(), colLast.data(), r);
                first = false;
                std::fill(rowA.begin(), rowA.end(), 0);
                std::fill(colA.begin(), colA.end(), 0);
                std::fill(colRow.begin(), colRow.end(), n);
                numAssigned = 0;
                assignmentPerRow.assign(n, n);
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
            }
            dense_zero_pass = true;
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
            lastRounds++;
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
