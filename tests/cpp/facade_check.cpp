// facade_check.cpp — compiles the C++ facade (include/tbdk.hpp) against
// libtbdk.so and exercises its host-only paths.  Exit code 0 = pass.
//   no GPU : Context throws tbdk::Error(TBDK_ENODEV) — the product path fails loudly
//   GPU    : a small pyramid + LK + GFTT + warp round trip through the facade
#include <cstdio>
#include <cstring>
#include <vector>

#include <hip/hip_runtime.h>

#include "tbdk.hpp"

int main(int argc, char** argv)
{
    const bool want_gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
    std::printf("%s\n", tbdk_version());
    tbdk_tbd_config cfg = tbdk::TbdLoop::defaultConfig(1920, 1080);
    if (cfg.win != 21 || cfg.max_level != 2 || cfg.bounds_xmax != 1280) return 2;
    try {
        tbdk::Context ctx(0);
        if (!want_gpu) return 3;  // a context without a GPU must not exist
        const int W = 320, H = 240;
        std::vector<uint8_t> h((size_t)W * H);
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) h[(size_t)y * W + x] = (uint8_t)((x * 7 + y * 13 + ((x / 9) ^ (y / 7)) * 40) & 255);
        uint8_t *d0, *d1;
        float *pts, *nxt, *corners;
        uint8_t* st;
        int32_t* cnt;
        if (hipMalloc(&d0, h.size()) || hipMalloc(&d1, h.size()) || hipMalloc(&pts, 8 * 64) ||
            hipMalloc(&nxt, 8 * 64) || hipMalloc(&st, 64) || hipMalloc(&corners, 8 * 64) || hipMalloc(&cnt, 4))
            return 4;
        (void)hipMemcpy(d0, h.data(), h.size(), hipMemcpyHostToDevice);
        tbdk::GpuImage a{d0, W, H, W}, b{d1, W, H, W};
        const double M[6] = {1, 0, 1.5, 0, 1, -0.5};  // b = a shifted by (1.5, -0.5)
        tbdk::cuda::warpAffine(ctx, a, b, M, TBDK_INTER_LINEAR, TBDK_BORDER_REFLECT_101);
        auto det = tbdk::cuda::CornersDetector::create(ctx, 64, 0.01, 5.0);
        det->detect(a, corners, cnt);
        int n = 0;
        (void)hipMemcpy(&n, cnt, 4, hipMemcpyDeviceToHost);
        if (n <= 0) return 5;
        (void)hipMemcpy(pts, corners, 8 * (size_t)n, hipMemcpyDeviceToDevice);
        auto lk = tbdk::cuda::SparsePyrLKOpticalFlow::create(ctx, {21, 21}, 2);
        lk->calc(a, b, pts, nxt, st, nullptr, n);
        std::vector<float> p0(2 * n), p1(2 * n);
        std::vector<uint8_t> s(n);
        (void)hipMemcpy(p0.data(), pts, 8 * (size_t)n, hipMemcpyDeviceToHost);
        (void)hipMemcpy(p1.data(), nxt, 8 * (size_t)n, hipMemcpyDeviceToHost);
        (void)hipMemcpy(s.data(), st, n, hipMemcpyDeviceToHost);
        int good = 0;
        for (int i = 0; i < n; ++i)
            if (s[i] && std::abs(p1[2 * i] - p0[2 * i] - 1.5f) < 0.1f && std::abs(p1[2 * i + 1] - p0[2 * i + 1] + 0.5f) < 0.1f)
                ++good;
        std::printf("corners %d tracked-correctly %d\n", n, good);
        if (good * 10 < n * 8) return 6;
        {  // the fp16 pixel path through the facade: fp16 pyramids from the u8 frames
            tbdk::Pyramid P(ctx, W, H, 2, {21, 21}, TBDK_DEPTH_16F), N(ctx, W, H, 2, {21, 21}, TBDK_DEPTH_16F);
            P.build(a);
            N.build(b);
            lk->calc(P, N, pts, nxt, st, nullptr, n);
            (void)hipMemcpy(p1.data(), nxt, 8 * (size_t)n, hipMemcpyDeviceToHost);
            (void)hipMemcpy(s.data(), st, n, hipMemcpyDeviceToHost);
            int good16 = 0;
            for (int i = 0; i < n; ++i)
                if (s[i] && std::abs(p1[2 * i] - p0[2 * i] - 1.5f) < 0.1f &&
                    std::abs(p1[2 * i + 1] - p0[2 * i + 1] + 0.5f) < 0.1f)
                    ++good16;
            std::printf("fp16 tracked-correctly %d\n", good16);
            if (good16 * 10 < n * 8 || P.depth() != TBDK_DEPTH_16F) return 7;
        }
        {  // CV_32FC3 / CV_16UC4 frames through the typed calc (the fp32 pixel path, cn channels)
            std::vector<uint8_t> hb((size_t)W * H);
            (void)hipMemcpy(hb.data(), d1, hb.size(), hipMemcpyDeviceToHost);
            std::vector<float> fa((size_t)W * H * 3), fb3((size_t)W * H * 3);
            std::vector<uint16_t> ua((size_t)W * H * 4), ub((size_t)W * H * 4);
            for (size_t k = 0; k < (size_t)W * H; ++k) {
                const float va = h[k], vb = hb[k];
                fa[3 * k] = va, fa[3 * k + 1] = 0.5f * va + 10.f, fa[3 * k + 2] = 255.f - va;
                fb3[3 * k] = vb, fb3[3 * k + 1] = 0.5f * vb + 10.f, fb3[3 * k + 2] = 255.f - vb;
                for (int c = 0; c < 4; ++c) {
                    ua[4 * k + c] = (uint16_t)(h[k] * 257 / (c + 1));
                    ub[4 * k + c] = (uint16_t)(hb[k] * 257 / (c + 1));
                }
            }
            void *dfa, *dfb, *dua, *dub;
            if (hipMalloc(&dfa, fa.size() * 4) || hipMalloc(&dfb, fb3.size() * 4) || hipMalloc(&dua, ua.size() * 2) ||
                hipMalloc(&dub, ub.size() * 2))
                return 4;
            (void)hipMemcpy(dfa, fa.data(), fa.size() * 4, hipMemcpyHostToDevice);
            (void)hipMemcpy(dfb, fb3.data(), fb3.size() * 4, hipMemcpyHostToDevice);
            (void)hipMemcpy(dua, ua.data(), ua.size() * 2, hipMemcpyHostToDevice);
            (void)hipMemcpy(dub, ub.data(), ub.size() * 2, hipMemcpyHostToDevice);
            const tbdk::GpuMatView views[2][2] = {
                {{dfa, W, H, W * 12, tbdk::DEPTH_32F, 3}, {dfb, W, H, W * 12, tbdk::DEPTH_32F, 3}},
                {{dua, W, H, W * 8, tbdk::DEPTH_16U, 4}, {dub, W, H, W * 8, tbdk::DEPTH_16U, 4}}};
            for (int t = 0; t < 2; ++t) {
                lk->calc(views[t][0], views[t][1], pts, nxt, st, nullptr, n);
                (void)hipMemcpy(p1.data(), nxt, 8 * (size_t)n, hipMemcpyDeviceToHost);
                (void)hipMemcpy(s.data(), st, n, hipMemcpyDeviceToHost);
                int goodc = 0;
                for (int i = 0; i < n; ++i)
                    if (s[i] && std::abs(p1[2 * i] - p0[2 * i] - 1.5f) < 0.1f &&
                        std::abs(p1[2 * i + 1] - p0[2 * i + 1] + 0.5f) < 0.1f)
                        ++goodc;
                std::printf("%s tracked-correctly %d\n", t == 0 ? "32FC3" : "16UC4", goodc);
                if (goodc * 10 < n * 8) return 12;
            }
        }
        // dense Farneback through the facade: the interior flow is the shift
        float* flow;
        if (hipMalloc(&flow, (size_t)W * H * 8)) return 4;
        auto fb = tbdk::cuda::FarnebackOpticalFlow::create(ctx);
        fb->calc(a, b, flow, W * 8);
        std::vector<float> fl((size_t)W * H * 2);
        (void)hipMemcpy(fl.data(), flow, fl.size() * 4, hipMemcpyDeviceToHost);
        int near = 0, tot = 0;
        for (int y = 40; y < H - 40; ++y)
            for (int x = 40; x < W - 40; ++x, ++tot) {
                const float* f = &fl[((size_t)y * W + x) * 2];
                near += std::abs(f[0] - 1.5f) < 0.25f && std::abs(f[1] + 0.5f) < 0.25f;
            }
        std::printf("farneback interior near-shift %d / %d\n", near, tot);
        if (near * 10 < tot * 8) return 8;
        // dense PyrLK through the facade
        auto dlk = tbdk::cuda::DensePyrLKOpticalFlow::create(ctx);
        dlk->calc(a, b, flow, W * 8);
        (void)hipMemcpy(fl.data(), flow, fl.size() * 4, hipMemcpyDeviceToHost);
        near = 0;
        for (int y = 40; y < H - 40; ++y)
            for (int x = 40; x < W - 40; ++x) {
                const float* f = &fl[((size_t)y * W + x) * 2];
                near += std::abs(f[0] - 1.5f) < 0.25f && std::abs(f[1] + 0.5f) < 0.25f;
            }
        std::printf("dense pyrlk interior near-shift %d / %d\n", near, tot);
        if (near * 10 < tot * 6) return 9;
        // HOG through the facade: every window of a gray frame scored, grouped
        auto hog = tbdk::cuda::HOG::create(ctx, {48, 96});
        std::vector<float> svm(hog->getDescriptorSize() + 1, 0.f);
        svm.back() = 1.f;  // bias only: every window scores 1 >= the hit threshold
        hog->setSVMDetector(svm);
        hog->setNumLevels(3);
        std::vector<double> conf;
        const auto rects = hog->detectMultiScale(a, 1, &conf);
        std::printf("hog rects %zu\n", rects.size());
        if (rects.empty() || conf.size() != rects.size() || conf[0] != 1.0) return 10;
        // ungrouped, stride 4: more hits than the first result buffer (4096) holds
        hog->setGroupThreshold(0);
        hog->setWinStride({4, 4});
        const auto all = hog->detectMultiScale(a, 1, &conf);
        std::printf("hog ungrouped %zu\n", all.size());
        return all.size() > 4096 && conf.size() == all.size() ? 0 : 11;
    } catch (const tbdk::Error& e) {
        std::printf("tbdk::Error: %s\n", e.what());
        return (!want_gpu && e.code() == TBDK_ENODEV) ? 0 : 7;
    }
}
