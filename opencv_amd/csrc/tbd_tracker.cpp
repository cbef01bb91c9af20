// tbd_tracker.cpp — see tbd_tracker.hpp.  Every function cites the reference
// function (modules/trackingbydetection/src/tbd.cpp) whose behaviour it restates.
#include "tbd_tracker.hpp"

#include <algorithm>
#include <cmath>
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
    for (auto& t : tracks) {
        const Rect& bbox = t.bboxes.back();
        double cx, cy;
        const Prediction* p = nullptr;
        for (int k = 0; preds && k < npreds; ++k)
            if (preds[k].id == t.id && preds[k].valid) {
                p = &preds[k];
                break;
            }
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
    std::vector<Track> kept;
    kept.reserve(tracks.size());
    for (auto& t : tracks) {
        const Rect& r = t.predPosition;
        if (r.x + r.width < xmin || r.x >= xmax || r.y + r.height < ymin || r.y >= ymax)
            deletedIds.push_back(t.id);
        else
            kept.push_back(std::move(t));
    }
    tracks.swap(kept);
}

// calculateCostMatrix + solveAssignmentProblem + classifyAssignments
// (tbd.cpp:333-891), flat n x n matrix, zero pattern cached per outer round
void Tracker::solveAssignment(std::vector<Detection>& dets, std::vector<int>& assignments,
                              std::vector<unsigned>& unassignedTracks, std::vector<unsigned>& unassignedDetections)
{
    const unsigned nT = (unsigned)tracks.size(), nD = (unsigned)dets.size();
    const unsigned n = std::max(nT, nD);
    const double huge = 10000000.0;
    const double pad = args.costOfNonAssignment * 2;
    cost.assign((size_t)n * n, pad);
    for (unsigned i = 0; i < nT; ++i)
        for (unsigned j = 0; j < nD; ++j)
            cost[(size_t)i * n + j] = 1.0 - computeBoundingBoxOverlap(tracks[i].predPosition, dets[j].bbox);
    assignmentPerRow.assign(n, n);
    auto C = [&](unsigned r, unsigned c) -> double& { return cost[(size_t)r * n + c]; };

    if (n > 0) {
        // step 1: row minima (tbd.cpp:494-516)
        for (unsigned r = 0; r < n; ++r) {
            double m = huge;
            for (unsigned c = 0; c < n; ++c) m = (C(r, c) < m) ? C(r, c) : m;
            for (unsigned c = 0; c < n; ++c) C(r, c) -= m;
        }
        // step 2: column minima (:539-561)
        for (unsigned c = 0; c < n; ++c) {
            double m = huge;
            for (unsigned r = 0; r < n; ++r) m = (C(r, c) < m) ? C(r, c) : m;
            for (unsigned r = 0; r < n; ++r) C(r, c) -= m;
        }
        std::vector<uint8_t> zero((size_t)n * n);
        std::vector<unsigned> rowZeros(n), colZeros(n);
        std::vector<char> rowA(n), colA(n), rowM(n), colM(n), rowCov(n), colCov(n);
        while (true) {  // (:585-887)
            for (size_t k = 0; k < zero.size(); ++k) zero[k] = equalsZero(cost[k]) ? 1 : 0;
            std::fill(rowZeros.begin(), rowZeros.end(), 0u);
            std::fill(colZeros.begin(), colZeros.end(), 0u);
            for (unsigned r = 0; r < n; ++r)
                for (unsigned c = 0; c < n; ++c)
                    if (zero[(size_t)r * n + c]) {
                        rowZeros[r]++;
                        colZeros[c]++;
                    }
            std::fill(rowA.begin(), rowA.end(), 0);
            std::fill(colA.begin(), colA.end(), 0);
            unsigned numAssigned = 0;
            assignmentPerRow.assign(n, n);
            bool made = true;
            while (made) {
                made = false;
                // rows with exactly one zero (:607-636)
                for (unsigned r = 0; r < n; ++r) {
                    if (rowA[r] || rowZeros[r] != 1) continue;
                    unsigned c = 0;
                    while (!zero[(size_t)r * n + c]) ++c;
                    if (!colA[c]) {
                        rowA[r] = colA[c] = 1;
                        assignmentPerRow[r] = c;
                        made = true;
                        numAssigned++;
                    }
                }
                // columns with exactly one zero (:639-668)
                for (unsigned c = 0; c < n; ++c) {
                    if (colA[c] || colZeros[c] != 1) continue;
                    unsigned r = 0;
                    while (!zero[(size_t)r * n + c]) ++r;
                    if (!rowA[r]) {
                        rowA[r] = colA[c] = 1;
                        assignmentPerRow[r] = c;
                        made = true;
                        numAssigned++;
                    }
                }
                // otherwise: first free zero of every unassigned row (:672-714)
                if (!made) {
                    for (unsigned r = 0; r < n; ++r) {
                        if (rowA[r]) continue;
                        for (unsigned c = 0; c < n; ++c) {
                            if (zero[(size_t)r * n + c] && !colA[c]) {
                                rowA[r] = colA[c] = 1;
                                assignmentPerRow[r] = c;
                                made = true;
                                numAssigned++;
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
                    for (unsigned c = 0; c < n; ++c)
                        if (zero[(size_t)r * n + c] && !colM[c]) {
                            colM[c] = 1;
                            newly++;
                        }
                }
                for (unsigned c = 0; c < n; ++c) {
                    if (!colM[c]) continue;
                    for (unsigned r2 = 0; r2 < n; ++r2)
                        if (assignmentPerRow[r2] == c) rowM[r2] = 1;
                }
                if (newly == 0) break;
            }
            bool allMarked = true;
            for (unsigned r = 0; r < n; ++r) {
                rowCov[r] = !rowM[r];
                if (!rowM[r]) allMarked = false;
            }
            if (allMarked) break;
            for (unsigned c = 0; c < n; ++c) colCov[c] = colM[c];
            // step 4 (:853-886)
            double mu = huge;
            for (unsigned r = 0; r < n; ++r) {
                if (rowCov[r]) continue;
                for (unsigned c = 0; c < n; ++c) {
                    if (colCov[c]) continue;
                    mu = (C(r, c) < mu) ? C(r, c) : mu;
                }
            }
            for (unsigned r = 0; r < n; ++r)
                for (unsigned c = 0; c < n; ++c) {
                    if (!rowCov[r] && !colCov[c]) C(r, c) -= mu;
                    else if (rowCov[r] && colCov[c]) C(r, c) += mu;
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
    for (unsigned k = (unsigned)t.scores.size() - num; k < t.scores.size(); ++k) {
        const double s = t.scores[k];
        sum += s;
        if (s > maxScore) maxScore = s;
    }
    t.maxConfidence = maxScore;
    t.avgConfidence = sum / num;
}

static void push_box(Track& t, const Rect& r, int frame, double score, unsigned window)
{
    t.bboxes.push_back(r);
    if (t.bboxes.size() > 4) t.bboxes.pop_front();
    t.frames.push_back(frame);
    if (t.frames.size() > 2) t.frames.pop_front();
    t.scores.push_back(score);
    if (t.scores.size() > window) t.scores.pop_front();
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
        for (size_t k = t.bboxes.size() - nprior; k < t.bboxes.size(); ++k) {
            wsum += t.bboxes[k].width;
            hsum += t.bboxes[k].height;
        }
        const int w = (wsum + d.bbox.width) / (nprior + 1);
        const int h = (hsum + d.bbox.height) / (nprior + 1);
        double cx = d.bbox.x, cy = d.bbox.y;
        cx += (d.bbox.width / 2) - (w / 2);
        cy += (d.bbox.height / 2) - (h / 2);
        t.bboxOverlap = computeBoundingBoxOverlap(d.bbox, t.predPosition);
        push_box(t, rect_from_point2d(cx, cy, w, h), d.frame_id, d.confidence, args.timeWindowSize);
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
        push_box(t, t.predPosition, frame_id, 0.0, args.timeWindowSize);
        t.bboxOverlap = 0.0;
        updateTrackConfidence(t);
    }
}

// deleteLostTracks (tbd.cpp:1011-1037)
void Tracker::deleteLostTracks()
{
    std::vector<Track> kept;
    kept.reserve(tracks.size());
    for (auto& t : tracks) {
        const double visibility = ((double)t.totalVisibleCount) / t.age;
        if ((t.age <= args.trackAgeThreshold && visibility <= args.trackVisibilityThreshold) ||
            (t.maxConfidence >= 0.0 && t.maxConfidence <= args.trackConfidenceThreshold))
            deletedIds.push_back(t.id);
        else
            kept.push_back(std::move(t));
    }
    tracks.swap(kept);
}

// createNewTracks + Track::Track(Detection&, Tracker*) (tbd.cpp:1043-1055, 67-91);
// the display colour drawn from rand() (:71-74) is not reproduced
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
        createdIds.push_back(t.id);
        tracks.push_back(std::move(t));
    }
}

// performTrackingStep (tbd.cpp:210-286)
void Tracker::performTrackingStep(std::vector<Detection>& dets, int frame_id, const Prediction* preds, int npreds)
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
    for (size_t i = 0; i < tracks.size(); ++i)
        if (assignments[i] >= 0) numAssigned++;
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
