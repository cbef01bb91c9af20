// synth.hip — renders the deterministic synthetic TBD sequence (synth_spec.h)
// directly into HBM, so benchmark frames are resident before timing starts.
#include "synth_spec.h"
#include "tbdk_internal.hpp"

namespace tbdk {

__global__ void synth_kernel(const syn_pose* __restrict__ poses, int nobj, uint32_t bgseed, int W, int H,
                             uint8_t* __restrict__ out, int pitch)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int f = blockIdx.z;
    if (x >= W) return;
    const syn_pose* fp = poses + (size_t)f * nobj;
    out[((size_t)f * H + y) * pitch + x] = syn_pixel(fp, nobj, x, y, bgseed);
}

hipError_t launch_synth(const void* poses_dev, int nobj, uint32_t bgseed, int W, int H, int nframes,
                        uint8_t* out, int pitch, hipStream_t s)
{
    dim3 block(256), grid((W + 255) / 256, H, nframes);
    hipLaunchKernelGGL(synth_kernel, grid, block, 0, s, static_cast<const syn_pose*>(poses_dev), nobj, bgseed, W,
                       H, out, pitch);
    return hipGetLastError();
}

// The HBM stream-copy peak for the bench's copy_peak denominator (SURVEY.md
// §8(d)): 16 bytes per lane (global_load_dwordx4 / global_store_dwordx4), four
// loads in flight per lane before the stores, consecutive lanes on consecutive
// 16-byte words, a grid of whole 4 KiB chunks per wave-quad.
constexpr int kCopyThreads = 256, kCopyUnroll = 4;

__global__ __launch_bounds__(kCopyThreads) void hbm_copy_kernel(const uint4* __restrict__ src,
                                                                uint4* __restrict__ dst, size_t n16)
{
    const size_t base = (size_t)blockIdx.x * (kCopyThreads * kCopyUnroll) + threadIdx.x;
    if (base + (size_t)(kCopyUnroll - 1) * kCopyThreads < n16) {
        uint4 v[kCopyUnroll];
#pragma unroll
        for (int k = 0; k < kCopyUnroll; ++k) v[k] = src[base + (size_t)k * kCopyThreads];
#pragma unroll
        for (int k = 0; k < kCopyUnroll; ++k) dst[base + (size_t)k * kCopyThreads] = v[k];
        return;
    }
    for (int k = 0; k < kCopyUnroll; ++k) {
        const size_t i = base + (size_t)k * kCopyThreads;
        if (i < n16) dst[i] = src[i];
    }
}

hipError_t launch_hbm_copy(const void* src, void* dst, size_t n16, hipStream_t s)
{
    const size_t per = (size_t)kCopyThreads * kCopyUnroll;
    const size_t blocks = (n16 + per - 1) / per;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(hbm_copy_kernel, dim3((unsigned)blocks), dim3(kCopyThreads), 0, s,
                       static_cast<const uint4*>(src), static_cast<uint4*>(dst), n16);
    return hipGetLastError();
}

}  // namespace tbdk
