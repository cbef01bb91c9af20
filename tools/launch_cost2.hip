// launch_cost2.hip -- host cost per launch of the TBD loop's kernel shapes by
// launch API: hipLaunchKernelGGL, hipModuleLaunchKernel on a function handle
// resolved once (hipGetFuncBySymbol, argument buffer via
// HIP_LAUNCH_PARAM_BUFFER_POINTER), hipExtLaunchKernel; argument structs of 64
// and 784 bytes (LkArgs); one stream, and round-robin over three streams.
// Build: hipcc --offload-arch=gfx950 -O2 tools/launch_cost2.hip -o tools/bin/launch_cost2
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

template <int B>
struct Args {
    int* p;
    int n;
    char pad[B - 12];
};
template <int B>
__global__ void k_args(Args<B> a)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n) a.p[i] += a.pad[i & 7];
}

int main()
{
    int* d = nullptr;
    (void)hipMalloc(&d, 1 << 20);
    hipStream_t s[3];
    for (auto& x : s) (void)hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
    const int N = 20000;
    using clk = std::chrono::steady_clock;
    auto per = [&](auto fn) {
        for (int i = 0; i < 300; ++i) fn(i);
        (void)hipDeviceSynchronize();
        auto t0 = clk::now();
        for (int i = 0; i < N; ++i) fn(i);
        auto t1 = clk::now();
        (void)hipDeviceSynchronize();
        return std::chrono::duration<double, std::micro>(t1 - t0).count() / N;
    };
    Args<64> a64;
    std::memset(&a64, 0, sizeof(a64));
    a64.p = d;
    a64.n = 1024;
    Args<784> a784;
    std::memset(&a784, 0, sizeof(a784));
    a784.p = d;
    a784.n = 1024;
    hipFunction_t f64 = nullptr, f784 = nullptr;
    (void)hipGetFuncBySymbol(&f64, reinterpret_cast<const void*>(&k_args<64>));
    (void)hipGetFuncBySymbol(&f784, reinterpret_cast<const void*>(&k_args<784>));
    auto mod = [&](hipFunction_t f, void* arg, size_t sz, hipStream_t st) {
        size_t size = sz;
        void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, arg, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
        (void)hipModuleLaunchKernel(f, 4, 1, 1, 256, 1, 1, 0, st, nullptr, cfg);
    };
    const double g64 = per([&](int) { hipLaunchKernelGGL(k_args<64>, dim3(4), dim3(256), 0, s[0], a64); });
    const double g784 = per([&](int) { hipLaunchKernelGGL(k_args<784>, dim3(4), dim3(256), 0, s[0], a784); });
    const double m64 = per([&](int) { mod(f64, &a64, sizeof(a64), s[0]); });
    const double m784 = per([&](int) { mod(f784, &a784, sizeof(a784), s[0]); });
    void* ea[] = {&a784};
    const double e784 = per([&](int) {
        (void)hipExtLaunchKernel(reinterpret_cast<const void*>(&k_args<784>), dim3(4), dim3(256), ea, 0, s[0], nullptr,
                                 nullptr, 0);
    });
    const double g784r = per([&](int i) { hipLaunchKernelGGL(k_args<784>, dim3(4), dim3(256), 0, s[i % 3], a784); });
    const double m784r = per([&](int i) { mod(f784, &a784, sizeof(a784), s[i % 3]); });
    std::printf("{\"ggl_64\": %.3f, \"ggl_784\": %.3f, \"module_64\": %.3f, \"module_784\": %.3f, \"ext_784\": %.3f, "
                "\"ggl_784_3streams\": %.3f, \"module_784_3streams\": %.3f, \"calls\": %d}\n",
                g64, g784, m64, m784, e784, g784r, m784r, N);
    return 0;
}
