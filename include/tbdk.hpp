// tbdk.hpp — header-only C++ facade over the C ABI (tbdk.h), shaped like the
// reference's cv::cuda interfaces for this path so a caller of
//   cv::cuda::SparsePyrLKOpticalFlow   (modules/cudaoptflow/include/opencv2/cudaoptflow.hpp:160-180)
//   cv::cuda::CornersDetector          (modules/cudaimgproc/include/opencv2/cudaimgproc.hpp:570-604)
//   cv::cuda::pyrDown / warpAffine     (modules/cudawarping/include/opencv2/cudawarping.hpp:126,201)
// changes types, not call structure.  Differences from the reference:
//   - images are non-owning device views (GpuImage) instead of GpuMat; the
//     caller owns all device memory;
//   - numerics follow the CPU reference (calcOpticalFlowPyrLK,
//     goodFeaturesToTrack, warpAffine), not the CUDA module's float variants;
//   - errors: tbdk::Error (a std::runtime_error carrying the TBDK_E* code)
//     where the reference throws cv::Exception.
#ifndef TBDK_HPP
#define TBDK_HPP

#include <cstdio>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "tbdk.h"

namespace tbdk {

class Error : public std::runtime_error {
public:
    Error(int code, const std::string& what) : std::runtime_error(what + ": " + name(code)), code_(code) {}
    int code() const { return code_; }
    static const char* name(int code)
    {
        switch (code) {
        case TBDK_EINVAL: return "TBDK_EINVAL (bad argument)";
        case TBDK_EHIP: return "TBDK_EHIP (HIP runtime error)";
        case TBDK_ENOMEM: return "TBDK_ENOMEM (device allocation failed)";
        case TBDK_ENODEV: return "TBDK_ENODEV (no such device)";
        default: return "unknown status";
        }
    }

private:
    int code_;
};

inline void check(int rc, const char* what)
{
    if (rc != TBDK_OK) throw Error(rc, what);
}

struct Size {
    int width = 0, height = 0;
};

// Non-owning device u8 image view (GpuMat of CV_8UC1 analogue).
struct GpuImage {
    uint8_t* data = nullptr;
    int width = 0, height = 0, pitch = 0;  // pitch in bytes
};

// Element depths of a typed view (cv::Mat depth codes): the types
// cv::cuda::SparsePyrLKOpticalFlow::calc accepts (cudaoptflow/src/pyrlk.cpp:189-205)
constexpr int DEPTH_8U = 0, DEPTH_16U = 2, DEPTH_32F = 5;

// Non-owning device image view with a depth and cn interleaved channels
// (GpuMat of CV_8UC1..4 / CV_16UC1..4 / CV_32FC1..4 analogue)
struct GpuMatView {
    void* data = nullptr;
    int width = 0, height = 0, pitch = 0;  // pitch in bytes
    int depth = DEPTH_8U, cn = 1;
};

// One context per (host thread, device); owns GFTT scratch and timing records.
class Context {
public:
    explicit Context(int device = 0) { check(tbdk_ctx_create(device, &h_), "tbdk_ctx_create"); }
    ~Context() { tbdk_ctx_destroy(h_); }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    tbdk_ctx* get() const { return h_; }
    int device() const { return tbdk_ctx_device(h_); }

private:
    tbdk_ctx* h_ = nullptr;
};

// Padded pyramid with Scharr derivative planes (buildOpticalFlowPyramid with
// withDerivatives=true, video/src/lkpyramid.cpp:697-793); depth TBDK_DEPTH_16F
// gives the fp16 pixel path's pyramid (tbdk_pyr_create_f16).
class Pyramid {
public:
    // depth TBDK_DEPTH_8U or TBDK_DEPTH_32F (cn 1..4 channels, interleaved), TBDK_DEPTH_16F (one channel)
    Pyramid(Context& ctx, int width, int height, int max_level, Size win = {21, 21}, int depth = TBDK_DEPTH_8U,
            int cn = 1)
        : ctx_(&ctx)
    {
        if (cn != 1 && depth == TBDK_DEPTH_16F) throw Error(TBDK_EINVAL, "Pyramid: fp16 pyramids are one-channel");
        if (depth == TBDK_DEPTH_16F)
            check(tbdk_pyr_create_f16(ctx.get(), width, height, max_level, win.width, win.height, &p_),
                  "tbdk_pyr_create_f16");
        else if (depth == TBDK_DEPTH_32F && cn != 1)
            check(tbdk_pyr_create_f32_cn(ctx.get(), width, height, cn, max_level, win.width, win.height, &p_),
                  "tbdk_pyr_create_f32_cn");
        else if (depth == TBDK_DEPTH_32F)
            check(tbdk_pyr_create_f32(ctx.get(), width, height, max_level, win.width, win.height, &p_),
                  "tbdk_pyr_create_f32");
        else if (cn != 1)
            check(tbdk_pyr_create_cn(ctx.get(), width, height, cn, max_level, win.width, win.height, &p_),
                  "tbdk_pyr_create_cn");
        else
            check(tbdk_pyr_create(ctx.get(), width, height, max_level, win.width, win.height, &p_), "tbdk_pyr_create");
    }
    ~Pyramid() { tbdk_pyr_destroy(ctx_->get(), &p_); }
    Pyramid(const Pyramid&) = delete;
    Pyramid& operator=(const Pyramid&) = delete;
    void build(const GpuImage& img, void* stream = nullptr)
    {
        if (img.width != p_.lv[0].width || img.height != p_.lv[0].height) throw Error(TBDK_EINVAL, "Pyramid::build");
        check(tbdk_pyr_build(ctx_->get(), img.data, img.pitch, &p_, stream), "tbdk_pyr_build");
    }
    // fp16 frame (pitch in bytes) into an fp16 pyramid
    void build_f16(const uint16_t* data, int width, int height, int pitch, void* stream = nullptr)
    {
        if (width != p_.lv[0].width || height != p_.lv[0].height) throw Error(TBDK_EINVAL, "Pyramid::build_f16");
        check(tbdk_pyr_build_f16(ctx_->get(), data, pitch, &p_, stream), "tbdk_pyr_build_f16");
    }
    // 16U / 32F frames (pitch in bytes) into an fp32 pyramid (the CUDA class's other depths)
    void build_u16(const uint16_t* data, int width, int height, int pitch, void* stream = nullptr)
    {
        if (width != p_.lv[0].width || height != p_.lv[0].height) throw Error(TBDK_EINVAL, "Pyramid::build_u16");
        check(tbdk_pyr_build_u16(ctx_->get(), data, pitch, &p_, stream), "tbdk_pyr_build_u16");
    }
    void build_f32(const float* data, int width, int height, int pitch, void* stream = nullptr)
    {
        if (width != p_.lv[0].width || height != p_.lv[0].height) throw Error(TBDK_EINVAL, "Pyramid::build_f32");
        check(tbdk_pyr_build_f32(ctx_->get(), data, pitch, &p_, stream), "tbdk_pyr_build_f32");
    }
    // any typed view the pyramid takes: u8 into either depth, u16 / fp32 into fp32
    // pyramids, with the pyramid's channel count
    void build(const GpuMatView& img, void* stream = nullptr)
    {
        if (img.width != p_.lv[0].width || img.height != p_.lv[0].height || img.cn != channels())
            throw Error(TBDK_EINVAL, "Pyramid::build");
        if (img.depth == DEPTH_8U)
            check(tbdk_pyr_build(ctx_->get(), static_cast<const uint8_t*>(img.data), img.pitch, &p_, stream),
                  "tbdk_pyr_build");
        else if (img.depth == DEPTH_16U)
            check(tbdk_pyr_build_u16(ctx_->get(), static_cast<const uint16_t*>(img.data), img.pitch, &p_, stream),
                  "tbdk_pyr_build_u16");
        else if (img.depth == DEPTH_32F)
            check(tbdk_pyr_build_f32(ctx_->get(), static_cast<const float*>(img.data), img.pitch, &p_, stream),
                  "tbdk_pyr_build_f32");
        else
            throw Error(TBDK_EINVAL, "Pyramid::build: depth");
    }
    int depth() const { return p_.depth; }
    int channels() const { return p_.cn > 1 ? p_.cn : 1; }
    const tbdk_pyr& get() const { return p_; }
    int levels() const { return p_.nlevels; }

private:
    Context* ctx_;
    tbdk_pyr p_{};
};

namespace cuda {

// cv::cuda::SparsePyrLKOpticalFlow (cudaoptflow.hpp:160-180; impl pyrlk.cpp:301-350).
// Like the reference implementation object it caches the prev/next pyramids
// (prevPyr_/nextPyr_, pyrlk.cpp:101-102) and rebuilds them per calc() on images.
class SparsePyrLKOpticalFlow {
public:
    static std::unique_ptr<SparsePyrLKOpticalFlow> create(Context& ctx, Size winSize = {21, 21}, int maxLevel = 3,
                                                          int iters = 30, bool useInitialFlow = false)
    {
        return std::unique_ptr<SparsePyrLKOpticalFlow>(
            new SparsePyrLKOpticalFlow(ctx, winSize, maxLevel, iters, useInitialFlow));
    }

    Size getWinSize() const { return win_; }
    void setWinSize(Size s) { win_ = s; pyr_[0].reset(); pyr_[1].reset(); }
    int getMaxLevel() const { return max_level_; }
    void setMaxLevel(int v) { max_level_ = v; pyr_[0].reset(); pyr_[1].reset(); }
    int getNumIters() const { return iters_; }
    void setNumIters(int v) { iters_ = v; }
    bool getUseInitialFlow() const { return use_initial_flow_; }
    void setUseInitialFlow(bool v) { use_initial_flow_ = v; }
    // CPU-path extras (calcOpticalFlowPyrLK arguments): epsilon, flags, minEigThreshold
    void setEpsilon(double e) { eps_ = e; }
    void setMinEigThreshold(float t) { min_eig_ = t; }
    void setGetMinEigenvals(bool v) { min_eig_flag_ = v; }

    // calc(prevImg, nextImg, prevPts, nextPts, status, err, stream): all point
    // buffers are device arrays of n entries (float2 points, u8 status, f32 err);
    // err may be null (noArray()).
    void calc(const GpuImage& prevImg, const GpuImage& nextImg, const float* prevPts, float* nextPts,
              uint8_t* status, float* err, int n, void* stream = nullptr)
    {
        if (n == 0) return;  // reference: empty prevPts releases the outputs (pyrlk.cpp:221-227)
        for (int i = 0; i < 2; ++i) {
            const GpuImage& im = i == 0 ? prevImg : nextImg;
            if (!pyr_[i] || pyr_[i]->get().lv[0].width != im.width || pyr_[i]->get().lv[0].height != im.height ||
                pyr_[i]->depth() != TBDK_DEPTH_8U || pyr_[i]->channels() != 1)
                pyr_[i].reset(new Pyramid(*ctx_, im.width, im.height, max_level_, win_));
            pyr_[i]->build(im, stream);
        }
        calc(*pyr_[0], *pyr_[1], prevPts, nextPts, status, err, n, stream);
    }

    // Typed images (the CUDA class's accepted types, pyrlk.cpp:189-205): CV_8UC1..4
    // on the u8 path, CV_16UC1..4 / CV_32FC1..4 on the fp32 pixel path; both
    // images of one type.  The pyramids are cached per (size, depth, channels).
    void calc(const GpuMatView& prevImg, const GpuMatView& nextImg, const float* prevPts, float* nextPts,
              uint8_t* status, float* err, int n, void* stream = nullptr)
    {
        if (n == 0) return;
        if (prevImg.depth != nextImg.depth || prevImg.cn != nextImg.cn) throw Error(TBDK_EINVAL, "calc: types");
        // the CUDA class asserts cn 1, 3 or 4 on its frames (pyrlk.cpp:142,228);
        // prebuilt Pyramids (below) take any count, as calcOpticalFlowPyrLK does
        if (prevImg.cn != 1 && prevImg.cn != 3 && prevImg.cn != 4) throw Error(TBDK_EINVAL, "calc: channels");
        const int pdepth = prevImg.depth == DEPTH_8U ? TBDK_DEPTH_8U : TBDK_DEPTH_32F;
        for (int i = 0; i < 2; ++i) {
            const GpuMatView& im = i == 0 ? prevImg : nextImg;
            if (!pyr_[i] || pyr_[i]->get().lv[0].width != im.width || pyr_[i]->get().lv[0].height != im.height ||
                pyr_[i]->depth() != pdepth || pyr_[i]->channels() != im.cn)
                pyr_[i].reset(new Pyramid(*ctx_, im.width, im.height, max_level_, win_, pdepth, im.cn));
            pyr_[i]->build(im, stream);
        }
        calc(*pyr_[0], *pyr_[1], prevPts, nextPts, status, err, n, stream);
    }

    // Pyramids given explicitly (calcOpticalFlowPyrLK accepts prebuilt pyramids,
    // video/src/lkpyramid.cpp:1270-1324): the TBD loop reuses prev frame's.
    void calc(const Pyramid& prev, const Pyramid& next, const float* prevPts, float* nextPts, uint8_t* status,
              float* err, int n, void* stream = nullptr, int32_t* iters = nullptr)
    {
        tbdk_lk_params p;
        p.win_w = win_.width;
        p.win_h = win_.height;
        p.max_level = max_level_;
        p.max_count = iters_;
        p.epsilon = eps_;
        p.flags = (use_initial_flow_ ? TBDK_OPTFLOW_USE_INITIAL_FLOW : 0) |
                  (min_eig_flag_ ? TBDK_OPTFLOW_LK_GET_MIN_EIGENVALS : 0);
        p.min_eig_threshold = min_eig_;
        p.impl = 0;
        check(tbdk_lk_sparse(ctx_->get(), &prev.get(), &next.get(), prevPts, nextPts, status, err, iters, n, &p,
                             stream),
              "tbdk_lk_sparse");
    }

private:
    SparsePyrLKOpticalFlow(Context& ctx, Size win, int max_level, int iters, bool uif)
        : ctx_(&ctx), win_(win), max_level_(max_level), iters_(iters), use_initial_flow_(uif)
    {
    }
    Context* ctx_;
    Size win_;
    int max_level_, iters_;
    bool use_initial_flow_;
    double eps_ = 0.01;
    float min_eig_ = 1e-4f;
    bool min_eig_flag_ = false;
    std::unique_ptr<Pyramid> pyr_[2];
};

// cv::cuda::DensePyrLKOpticalFlow (cudaoptflow.hpp:182-208; impl pyrlk.cpp:238-299,
// 352-397): the PyrLK of every level-0 pixel, written as a CV_32FC2 flow field.
// useInitialFlow is kept for the interface and, as in the reference, has no effect.
class DensePyrLKOpticalFlow {
public:
    static std::unique_ptr<DensePyrLKOpticalFlow> create(Context& ctx, Size winSize = {13, 13}, int maxLevel = 3,
                                                         int iters = 30, bool useInitialFlow = false)
    {
        return std::unique_ptr<DensePyrLKOpticalFlow>(
            new DensePyrLKOpticalFlow(ctx, winSize, maxLevel, iters, useInitialFlow));
    }

    Size getWinSize() const { return win_; }
    void setWinSize(Size s) { win_ = s; pyr_[0].reset(); pyr_[1].reset(); }
    int getMaxLevel() const { return max_level_; }
    void setMaxLevel(int v) { max_level_ = v; pyr_[0].reset(); pyr_[1].reset(); }
    int getNumIters() const { return iters_; }
    void setNumIters(int v) { iters_ = v; }
    bool getUseInitialFlow() const { return use_initial_flow_; }
    void setUseInitialFlow(bool v) { use_initial_flow_ = v; }

    // calc(I0, I1, flow, stream): flow is a device CV_32FC2 image (flowPitch bytes
    // per row); status, when given, is a device u8 plane of statusPitch bytes per row.
    void calc(const GpuImage& I0, const GpuImage& I1, float* flow, int flowPitch, void* stream = nullptr,
              uint8_t* status = nullptr, int statusPitch = 0)
    {
        for (int i = 0; i < 2; ++i) {
            const GpuImage& im = i == 0 ? I0 : I1;
            if (!pyr_[i] || pyr_[i]->get().lv[0].width != im.width || pyr_[i]->get().lv[0].height != im.height)
                pyr_[i].reset(new Pyramid(*ctx_, im.width, im.height, max_level_, win_));
            pyr_[i]->build(im, stream);
        }
        tbdk_lk_params p;
        p.win_w = win_.width;
        p.win_h = win_.height;
        p.max_level = max_level_;
        p.max_count = iters_;
        p.epsilon = 0.01;
        p.flags = use_initial_flow_ ? TBDK_OPTFLOW_USE_INITIAL_FLOW : 0;
        p.min_eig_threshold = 1e-4f;
        p.impl = 0;
        check(tbdk_lk_dense(ctx_->get(), &pyr_[0]->get(), &pyr_[1]->get(), flow, flowPitch, status, statusPitch, &p,
                            stream),
              "tbdk_lk_dense");
    }

private:
    DensePyrLKOpticalFlow(Context& ctx, Size win, int max_level, int iters, bool uif)
        : ctx_(&ctx), win_(win), max_level_(max_level), iters_(iters), use_initial_flow_(uif)
    {
    }
    Context* ctx_;
    Size win_;
    int max_level_, iters_;
    bool use_initial_flow_;
    std::unique_ptr<Pyramid> pyr_[2];
};

// cv::cuda::CornersDetector from createGoodFeaturesToTrackDetector(CV_8UC1,
// maxCorners, qualityLevel, minDistance, blockSize=3, useHarris=false, harrisK=0.04)
// (cudaimgproc.hpp:582,603-604).  detect() runs on the whole image; detectRois()
// is the batched per-box form the TBD loop uses (one launch set for all boxes).
class CornersDetector {
public:
    static std::unique_ptr<CornersDetector> create(Context& ctx, int maxCorners = 1000, double qualityLevel = 0.01,
                                                   double minDistance = 0.0, int blockSize = 3,
                                                   bool useHarrisDetector = false, double harrisK = 0.04)
    {
        if (blockSize < 1 || blockSize > 63) throw Error(TBDK_EINVAL, "createGoodFeaturesToTrackDetector");
        return std::unique_ptr<CornersDetector>(
            new CornersDetector(ctx, maxCorners, qualityLevel, minDistance, blockSize, useHarrisDetector, harrisK));
    }

    // corners: device, maxCorners float2; count: device int32 (corners found, -1 on
    // candidate overflow).  The count stays on the device (no host sync).
    void detect(const GpuImage& image, float* corners, int32_t* count, void* stream = nullptr)
    {
        tbdk_roi r{0, 0, image.width, image.height};
        detectRois(image, &r, 1, corners, count, stream);
    }

    // rois: host array; corners: device nroi x maxCorners float2; counts: device nroi int32
    void detectRois(const GpuImage& image, const tbdk_roi* rois, int nroi, float* corners, int32_t* counts,
                    void* stream = nullptr)
    {
        check(tbdk_gftt_rois(ctx_->get(), image.data, image.width, image.height, image.pitch, rois, nroi, &p_,
                             corners, counts, stream),
              "tbdk_gftt_rois");
    }

private:
    CornersDetector(Context& ctx, int maxc, double q, double md, int block, bool harris, double k) : ctx_(&ctx)
    {
        p_.max_corners = maxc;
        p_.quality_level = q;
        p_.min_distance = md;
        p_.block_size = block;
        p_.use_harris = harris ? 1 : 0;
        p_.harris_k = k;
    }
    Context* ctx_;
    tbdk_gftt_params p_{};
};

// cv::cuda::createMinEigenValCorner(CV_8UC1, blockSize, 3)->compute (harris false) and
// cv::cuda::createHarrisCorner(CV_8UC1, blockSize, 3, k)->compute (harris true)
// (cudaimgproc.hpp:548-566): dst is a device float plane (dst_pitch bytes)
inline void cornerResponse(Context& ctx, const GpuImage& src, float* dst, int dst_pitch, int blockSize = 3,
                           bool harris = false, double k = 0.04, void* stream = nullptr)
{
    check(tbdk_corner_response(ctx.get(), src.data, src.width, src.height, src.pitch, dst, dst_pitch, blockSize,
                               harris ? 1 : 0, k, stream),
          "tbdk_corner_response");
}

// cv::cuda::pyrDown (cudawarping.hpp:201): dst must be ((w+1)/2, (h+1)/2)
inline void pyrDown(Context& ctx, const GpuImage& src, GpuImage& dst, void* stream = nullptr)
{
    if (dst.width != (src.width + 1) / 2 || dst.height != (src.height + 1) / 2) throw Error(TBDK_EINVAL, "pyrDown");
    check(tbdk_pyr_down_u8(ctx.get(), src.data, src.width, src.height, src.pitch, dst.data, dst.pitch, stream),
          "tbdk_pyr_down_u8");
}

// cv::cuda::warpAffine(src, dst, M, dsize, flags, borderMode, borderValue, stream)
// (cudawarping.hpp:126); dsize is dst's size; M is a host 2x3 row-major matrix.
inline void warpAffine(Context& ctx, const GpuImage& src, GpuImage& dst, const double M[6],
                       int flags = TBDK_INTER_LINEAR, int borderMode = TBDK_BORDER_CONSTANT, int borderValue = 0,
                       void* stream = nullptr)
{
    check(tbdk_warp_affine_u8(ctx.get(), src.data, src.width, src.height, src.pitch, dst.data, dst.width,
                              dst.height, dst.pitch, M, flags, borderMode, borderValue, stream),
          "tbdk_warp_affine_u8");
}

// cv::cuda::FarnebackOpticalFlow (cudaoptflow.hpp:210-252): create() with the
// reference's defaults, the getters/setters, calc(I0, I1, flow, stream).
// flow: device CV_32FC2 (dx, dy interleaved), flowPitch in bytes.
class FarnebackOpticalFlow {
public:
    static std::unique_ptr<FarnebackOpticalFlow> create(Context& ctx, int numLevels = 5, double pyrScale = 0.5,
                                                        bool fastPyramids = false, int winSize = 13,
                                                        int numIters = 10, int polyN = 5, double polySigma = 1.1,
                                                        int flags = 0)
    {
        std::unique_ptr<FarnebackOpticalFlow> f(new FarnebackOpticalFlow(ctx));
        f->p_ = tbdk_farneback_params{numLevels, pyrScale, fastPyramids ? 1 : 0, winSize, numIters, polyN,
                                      polySigma, flags};
        return f;
    }
    int getNumLevels() const { return p_.num_levels; }
    void setNumLevels(int v) { p_.num_levels = v; }
    double getPyrScale() const { return p_.pyr_scale; }
    void setPyrScale(double v) { p_.pyr_scale = v; }
    bool getFastPyramids() const { return p_.fast_pyramids != 0; }
    void setFastPyramids(bool v) { p_.fast_pyramids = v ? 1 : 0; }
    int getWinSize() const { return p_.win_size; }
    void setWinSize(int v) { p_.win_size = v; }
    int getNumIters() const { return p_.num_iters; }
    void setNumIters(int v) { p_.num_iters = v; }
    int getPolyN() const { return p_.poly_n; }
    void setPolyN(int v) { p_.poly_n = v; }
    double getPolySigma() const { return p_.poly_sigma; }
    void setPolySigma(double v) { p_.poly_sigma = v; }
    int getFlags() const { return p_.flags; }
    void setFlags(int v) { p_.flags = v; }

    void calc(const GpuImage& I0, const GpuImage& I1, float* flow, int flowPitch, void* stream = nullptr)
    {
        if (I0.width != I1.width || I0.height != I1.height || I0.pitch != I1.pitch)
            throw Error(TBDK_EINVAL, "FarnebackOpticalFlow::calc");
        check(tbdk_farneback(ctx_->get(), I0.data, I1.data, I0.width, I0.height, I0.pitch, flow, flowPitch, &p_,
                             stream),
              "tbdk_farneback");
    }

private:
    explicit FarnebackOpticalFlow(Context& ctx) : ctx_(&ctx) {}
    Context* ctx_;
    tbdk_farneback_params p_{};
};

}  // namespace cuda

namespace cuda {

// cv::cuda::HOG (cudaobjdetect.hpp:75-180) with the CPU HOGDescriptor's results
// (objdetect/src/hog.cpp): create / setters / setSVMDetector / detectMultiScale.
// Detector coefficients stay on the host; getDefaultPeopleDetector's tables ship
// as opencv_amd/data/hog_people_{64x128,48x96}.f32 (loadDetector reads them).
class HOG {
public:
    static std::unique_ptr<HOG> create(Context& ctx, Size winSize = {64, 128}, Size blockSize = {16, 16},
                                       Size blockStride = {8, 8}, Size cellSize = {8, 8}, int nbins = 9)
    {
        std::unique_ptr<HOG> h(new HOG(ctx));
        tbdk_hog_default_params(&h->p_);
        h->p_.win_w = winSize.width, h->p_.win_h = winSize.height;
        h->p_.block_w = blockSize.width, h->p_.block_h = blockSize.height;
        h->p_.block_stride_x = blockStride.width, h->p_.block_stride_y = blockStride.height;
        h->p_.cell_w = cellSize.width, h->p_.cell_h = cellSize.height;
        h->p_.nbins = nbins;
        h->p_.win_stride_x = blockStride.width, h->p_.win_stride_y = blockStride.height;
        h->getDescriptorSize();  // throws on an invalid geometry (HOG_Impl's asserts)
        return h;
    }
    void setGammaCorrection(bool v) { p_.gamma_correction = v; }
    void setL2HysThreshold(double v) { p_.l2hys_threshold = v; }
    void setNumLevels(int v) { p_.nlevels = v; }
    int getNumLevels() const { return p_.nlevels; }
    void setHitThreshold(double v) { p_.hit_threshold = v; }
    double getHitThreshold() const { return p_.hit_threshold; }
    void setWinStride(Size s) { p_.win_stride_x = s.width, p_.win_stride_y = s.height; }
    void setScaleFactor(double v) { p_.scale0 = v; }
    double getScaleFactor() const { return p_.scale0; }
    void setGroupThreshold(int v) { p_.group_threshold = v; }
    int getGroupThreshold() const { return p_.group_threshold; }
    void setWinSigma(double v) { p_.win_sigma = v; }
    int getDescriptorSize() const
    {
        int n = 0;
        check(tbdk_hog_descriptor_size(&p_, &n), "HOG: invalid geometry");
        return n;
    }
    void setSVMDetector(const std::vector<float>& d)
    {
        const size_t n = (size_t)getDescriptorSize();
        if (d.size() != n && d.size() != n + 1) throw Error(TBDK_EINVAL, "HOG::setSVMDetector");
        svm_ = d;
    }
    // reads one of the shipped detector tables (little-endian float32)
    static std::vector<float> loadDetector(const char* path)
    {
        std::vector<float> v;
        if (FILE* f = std::fopen(path, "rb")) {
            float x;
            while (std::fread(&x, 4, 1, f) == 1) v.push_back(x);
            std::fclose(f);
        }
        if (v.empty()) throw Error(TBDK_EINVAL, "HOG::loadDetector");
        return v;
    }
    // img: device u8, 1 (gray), 3 (BGR) or 4 (BGRA) channels; returns (x, y, w, h) rects
    std::vector<tbdk_roi> detectMultiScale(const GpuImage& img, int channels, std::vector<double>* confidences = nullptr,
                                           void* stream = nullptr)
    {
        std::vector<int32_t> r;
        std::vector<double> w;
        int n = 0;
        for (int cap = 4096;; cap *= 4) {  // grow and call again while the results overflow
            r.resize(4 * (size_t)cap);
            w.resize(cap);
            const int rc = tbdk_hog_detect_multiscale(ctx_->get(), img.data, img.width, img.height, img.pitch,
                                                      channels, &p_, svm_.data(), (int)svm_.size(), r.data(),
                                                      w.data(), cap, &n, stream);
            if (rc == TBDK_ENOMEM && n == cap) continue;
            check(rc, "tbdk_hog_detect_multiscale");
            break;
        }
        std::vector<tbdk_roi> out(n);
        for (int i = 0; i < n; ++i) out[i] = tbdk_roi{r[4 * i], r[4 * i + 1], r[4 * i + 2], r[4 * i + 3]};
        if (confidences) confidences->assign(w.begin(), w.begin() + n);
        return out;
    }

private:
    explicit HOG(Context& ctx) : ctx_(&ctx) {}
    Context* ctx_;
    tbdk_hog_params p_{};
    std::vector<float> svm_;
};

}  // namespace cuda


// The tracking section of samples/gpu/tbd.cpp:624-706 (cv::tbd::Tracker +
// KLT box propagation) for one video stream.
class TbdLoop {
public:
    TbdLoop(Context& ctx, const tbdk_tbd_config& cfg) { check(tbdk_tbd_create(ctx.get(), &cfg, &h_), "tbdk_tbd_create"); }
    ~TbdLoop() { tbdk_tbd_destroy(h_); }
    TbdLoop(const TbdLoop&) = delete;
    TbdLoop& operator=(const TbdLoop&) = delete;
    static tbdk_tbd_config defaultConfig(int width, int height)
    {
        tbdk_tbd_config c;
        check(tbdk_tbd_default_config(width, height, &c), "tbdk_tbd_default_config");
        return c;
    }
    tbdk_frame_metrics step(const GpuImage& frame, int frameId, const std::vector<tbdk_detection>& dets,
                            void* stream = nullptr)
    {
        tbdk_frame_metrics m;
        check(tbdk_tbd_step(h_, frame.data, frame.pitch, frameId, dets.data(), (int)dets.size(), &m, stream),
              "tbdk_tbd_step");
        return m;
    }
    std::vector<tbdk_track_info> tracks() const
    {
        std::vector<tbdk_track_info> out(4096);
        int n = 0;
        check(tbdk_tbd_tracks(h_, out.data(), (int)out.size(), &n), "tbdk_tbd_tracks");
        out.resize((size_t)(n < (int)out.size() ? n : (int)out.size()));
        return out;
    }

private:
    tbdk_tbd* h_ = nullptr;
};

}  // namespace tbdk

#endif  // TBDK_HPP
