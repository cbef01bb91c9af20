// gftt_probe.hip — standalone phase timing of the GFTT launches on the bench's
// frame-0 ground-truth boxes (1080p x 128 synthetic objects).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I include tools/gftt_probe.hip -o build/gftt_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__device__ unsigned long long* g_stamps;
#define GFTT_STAMP(i)                                                                   \
    do {                                                                                \
        if (threadIdx.x == 0) g_stamps[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
__device__ unsigned long long* g_estamps;
#define GFTT_ESTAMP(i)                                                                     \
    do {                                                                                   \
        if (threadIdx.x == 0) g_estamps[blockIdx.x * 4 + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
__device__ unsigned long long* g_tacc;
#define GFTT_TDECL                      \
    unsigned long long tacc_[6] = {0}; \
    unsigned long long tlast_ = 0;      \
    int tsteps_ = 0
#define GFTT_T(i)                                                        \
    do {                                                                 \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();       \
        if ((i) > 0) tacc_[(i)-1] += t_ - tlast_;                         \
        else tsteps_++;                                                  \
        tlast_ = t_;                                                     \
    } while (0)
#define GFTT_TDUMP                                                                  \
    do {                                                                            \
        if (threadIdx.x == 0) {                                                     \
            for (int q_ = 0; q_ < 5; ++q_) g_tacc[blockIdx.x * 8 + q_] = tacc_[q_]; \
            g_tacc[blockIdx.x * 8 + 5] = tsteps_;                                   \
        }                                                                           \
    } while (0)
#include "../opencv_amd/csrc/klt_gftt.hip"
#include "../opencv_amd/csrc/synth_spec.h"

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                      \
        }                                                                  \
    } while (0)

int main()
{
    const int W = 1920, H = 1080, N = 128;
    std::vector<syn_object> objs(N);
    syn_make_objects(20261015u, W, H, N, objs.data());
    std::vector<syn_pose> poses(N);
    for (int o = 0; o < N; ++o) syn_pose_at(&objs[o], W, H, 0, &poses[o]);
    std::vector<uint8_t> img((size_t)W * H);
    const uint32_t bg = syn_hash(20261015u ^ 0xB6A5EEDU);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) img[(size_t)y * W + x] = syn_pixel(poses.data(), N, x, y, bg);
    std::vector<tbdk::GfttRoi> rois;
    int total = 0, max_area = 0, max_w = 0, words = 0, ncblk = 0;
    for (int o = 0; o < N; ++o) {
        int32_t b[4];
        if (!syn_gt_box(&poses[o], W, H, b)) continue;
        rois.push_back(tbdk::GfttRoi{b[0], b[1], b[2], b[3], total, words, ncblk});
        if (b[2] >= 3 && b[3] >= 3) words += (b[2] + tbdk::kGfttStrip - 1) / tbdk::kGfttStrip * b[3];
        ncblk += (b[2] + tbdk::kGfttStrip - 1) / tbdk::kGfttStrip;
        total += tbdk::gftt_epitch(b[2]) * b[3];
        max_area = std::max(max_area, b[2] * b[3]);
        max_w = std::max(max_w, b[2]);
    }
    const int nroi = (int)rois.size();
    uint8_t* dimg;
    tbdk::GfttRoi* drois;
    double* planes;
    int *dmax, *dcc, *dcounts;  // per column-block max, per pixel-block count, per-ROI output
    void* dcand;
    float2* dcorners;
    unsigned long long* dst;
    CK(hipMalloc(&dimg, img.size()));
    CK(hipMemcpy(dimg, img.data(), img.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&drois, sizeof(tbdk::GfttRoi) * nroi));
    CK(hipMemcpy(drois, rois.data(), sizeof(tbdk::GfttRoi) * nroi, hipMemcpyHostToDevice));
    CK(hipMalloc(&planes, (sizeof(double) * 3 + 4) * (size_t)total));
    CK(hipMalloc(&dmax, 4 * ncblk));
    CK(hipMalloc(&dcc, 4));
    CK(hipMalloc(&dcounts, 4 * nroi));
    CK(hipMalloc(&dcand, 8 * (size_t)std::max(words, 1)));
    CK(hipMalloc(&dcorners, sizeof(float2) * 256 * nroi));
    CK(hipMalloc(&dst, 8 * 8 * nroi));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &dst, sizeof(dst)));
    unsigned long long* dest;
    CK(hipMalloc(&dest, 8 * 4 * (size_t)ncblk));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_estamps), &dest, sizeof(dest)));
    unsigned long long* dtacc;
    CK(hipMalloc(&dtacc, 8 * 8 * nroi));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_tacc), &dtacc, sizeof(dtacc)));
    tbdk::GfttArgs a{};
    a.img = dimg;
    a.pitch = W;
    a.rois = drois;
    a.nroi = nroi;
    a.ncblk = ncblk;
    a.eig = reinterpret_cast<float*>(planes);
    a.blk_max = dmax;
    a.lmax = static_cast<uint64_t*>(dcand);
    a.eig_redo = 0;
    a.max_corners = 256;
    a.quality = 0.01;
    a.min_distance = 3.0;
    a.corners = dcorners;
    a.counts = dcounts;
    tbdk::gftt_plan(a, max_area);
    printf("cap %d img_bytes %d\n", a.cap, a.img_bytes);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int it = 0; it < 5; ++it) CK(tbdk::launch_gftt(a, 0));
    CK(hipEventRecord(e0, 0));
    const int reps = 20;
    for (int it = 0; it < reps; ++it) CK(tbdk::launch_gftt(a, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> st(8 * nroi);
    std::vector<int> cnt(nroi);
    CK(hipMemcpy(st.data(), dst, 8 * 8 * nroi, hipMemcpyDeviceToHost));
    CK(hipMemcpy(cnt.data(), dcounts, 4 * nroi, hipMemcpyDeviceToHost));
    double ph[3] = {0, 0, 0}, pm[3] = {0, 0, 0};
    for (int r = 0; r < nroi; ++r)
        for (int k = 0; k < 3; ++k) {
            double d = (double)(st[8 * r + k + 1] - st[8 * r + k]);
            ph[k] += d / nroi;
            pm[k] = std::max(pm[k], d);
        }
    printf("nroi %d total px %d max_area %d: gftt %.1f us/launch\n", nroi, total, max_area, ms * 1000 / reps);
    {  // eigenvalue walk: per-workgroup spans of the last launch
        std::vector<unsigned long long> es(4 * (size_t)ncblk);
        CK(hipMemcpy(es.data(), dest, 8 * 4 * (size_t)ncblk, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull, t1 = 0;
        double walk = 0, wmax = 0, rest = 0;
        for (int b = 0; b < ncblk; ++b) {
            t0 = std::min(t0, es[4 * b]);
            t1 = std::max(t1, es[4 * b + 2]);
            const double w = (double)(es[4 * b + 1] - es[4 * b]);
            walk += w / ncblk;
            wmax = std::max(wmax, w);
            rest += (double)(es[4 * b + 2] - es[4 * b + 1]) / ncblk;
        }
        unsigned long long late = 0;
        for (int b = 0; b < ncblk; ++b) late = std::max(late, es[4 * b] - t0);
        printf("eig: %d workgroups, span %llu ticks (last start +%llu), walk mean %.0f max %.0f, after-walk mean %.0f\n",
               ncblk, t1 - t0, late, walk, wmax, rest);
    }
    printf("select phases (s_memtime ticks) mean/max: load %.0f/%.0f sort %.0f/%.0f walk %.0f/%.0f\n", ph[0], pm[0],
           ph[1], pm[1], ph[2], pm[2]);
    {
        double g = 0, ps = 0;
        for (int r = 0; r < nroi; ++r) {
            g += (double)(st[8 * r + 4] - st[8 * r]) / nroi;
            ps += (double)(st[8 * r + 5] - st[8 * r + 4]) / nroi;
        }
        printf("  load = gather %.0f + partial selection %.0f + padding %.0f\n", g, ps, ph[0] - g - ps);
    }
    long sa = 0;
    for (int r = 0; r < nroi; ++r) sa += cnt[r];
    std::vector<unsigned long long> ta(8 * nroi);
    CK(hipMemcpy(ta.data(), dtacc, 8 * 8 * nroi, hipMemcpyDeviceToHost));
    double tm[6] = {0, 0, 0, 0, 0, 0};
    for (int r = 0; r < nroi; ++r)
        for (int q = 0; q < 6; ++q) tm[q] += (double)ta[8 * r + q] / nroi;
    printf("walk sub-phases mean ticks: write %.0f window %.0f ballot/resolve %.0f limit %.0f store %.0f; steps %.1f\n",
           tm[0], tm[1], tm[2], tm[3], tm[4], tm[5]);
    printf("accepted mean %.1f\n", (double)sa / nroi);
    return 0;
}
