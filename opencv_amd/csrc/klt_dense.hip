// klt_dense.hip — dense pyramidal Lucas-Kanade: cv::cuda::DensePyrLKOpticalFlow
// (cudaoptflow/include/opencv2/cudaoptflow.hpp:182-208, impl
// cudaoptflow/src/pyrlk.cpp:238-299, 352-391) as the CPU cv::calcOpticalFlowPyrLK
// (video/src/lkpyramid.cpp:1207-1377) evaluated at every pixel of the frame:
// the same LK kernels as tbdk_lk_sparse over the full pixel grid, then the
// flow u = nextPt.x - x, v = nextPt.y - y written as CV_32FC2.
//
// The CUDA module's dense kernel has no CPU counterpart (float pyrDown
// pyramids, texture bilinear, no minEig gate, its own stop rule); this entry
// point keeps the CPU semantics of the sparse path so that both LK forms of
// the library agree point for point.
#include "tbdk_internal.hpp"

namespace tbdk {

namespace {

// the pixel grid (x, y) of a w x h frame, one float2 per pixel
__global__ __launch_bounds__(256) void dense_grid_kernel(float2* pts, int w, int h)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x < w) pts[(size_t)y * w + x] = make_float2((float)x, (float)y);
}

// flow = next - grid; status copied into a pitched plane when asked for
__global__ __launch_bounds__(256) void dense_flow_kernel(const float2* next, const uint8_t* st, int w, int h,
                                                         float* flow, int flow_pitch, uint8_t* status,
                                                         int status_pitch)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= w) return;
    const size_t i = (size_t)y * w + x;
    const float2 p = next[i];
    *reinterpret_cast<float2*>(reinterpret_cast<uint8_t*>(flow) + (size_t)y * flow_pitch + 8 * (size_t)x) =
        make_float2(p.x - (float)x, p.y - (float)y);
    if (status) status[(size_t)y * status_pitch + x] = st[i];
}

}  // namespace

}  // namespace tbdk

using namespace tbdk;

extern "C" {

int tbdk_lk_dense(tbdk_ctx* ctx, const tbdk_pyr* prev, const tbdk_pyr* next, float* flow, int flow_pitch,
                  uint8_t* status, int status_pitch, const tbdk_lk_params* p, void* stream)
{
    if (!ctx || !prev || !next || !flow || !p || prev->nlevels <= 0) return TBDK_EINVAL;
    if (prev->cn > 1 || next->cn > 1) return TBDK_EINVAL;  // the dense path takes one-channel pyramids
    // CV_Assert(winSize_[0] > 2 && winSize_[1] > 2) of PyrLKOpticalFlowBase::dense (pyrlk.cpp:243)
    if (p->win_w <= 2 || p->win_h <= 2) return TBDK_EINVAL;
    // the reference's dense() never reads the incoming flow, so useInitialFlow has
    // no effect there (pyrlk.cpp:238-299): drop the flag rather than reject it
    tbdk_lk_params prm = *p;
    prm.flags &= ~TBDK_OPTFLOW_USE_INITIAL_FLOW;
    const int w = prev->lv[0].width, h = prev->lv[0].height;
    if (next->nlevels <= 0 || next->lv[0].width != w || next->lv[0].height != h) return TBDK_EINVAL;
    if (flow_pitch < 8 * w || flow_pitch % 8 != 0 || (status && status_pitch < w)) return TBDK_EINVAL;
    const int64_t n = (int64_t)w * h;
    if (n > INT32_MAX) return TBDK_EINVAL;
    DeviceGuard g(ctx->device);
    // scratch: grid points, next points (float2 each) and status per pixel
    if (n > ctx->dense_cap) {
        if (ctx->dense_buf) (void)hipFree(ctx->dense_buf);
        ctx->dense_buf = nullptr;
        ctx->dense_cap = 0;
        if (hipMalloc(&ctx->dense_buf, (size_t)n * 17 + 256) != hipSuccess) return TBDK_ENOMEM;
        ctx->dense_cap = n;
    }
    float2* pts = static_cast<float2*>(ctx->dense_buf);
    float2* nxt = pts + n;
    uint8_t* st = reinterpret_cast<uint8_t*>(nxt + n);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid((w + 255) / 256, h);
    hipLaunchKernelGGL(dense_grid_kernel, grid, dim3(256), 0, s, pts, w, h);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return map_status(e);
    const int rc = lk_internal(ctx, prev, next, reinterpret_cast<const float*>(pts), reinterpret_cast<float*>(nxt),
                               st, nullptr, nullptr, (int)n, &prm, nullptr, 0, stream);
    if (rc != TBDK_OK) return rc;
    hipLaunchKernelGGL(dense_flow_kernel, grid, dim3(256), 0, s, nxt, st, w, h, flow, flow_pitch, status,
                       status_pitch);
    return map_status(hipGetLastError());
}

}  // extern "C"
