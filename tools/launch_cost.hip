// launch_cost.hip -- host-side cost of the HIP calls the TBD loop makes per frame
// (hipLaunchKernelGGL of a small kernel, hipEventRecord, hipStreamWaitEvent,
// hipEventQuery), measured on the calling thread: mean microseconds per call over
// N calls, the device kept busy by nothing else.  Build: hipcc --offload-arch=gfx950
// -O2 tools/launch_cost.hip -o tools/bin/launch_cost
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void tiny(int* p, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += 1;
}

struct Args {
    const int* a;
    int* b;
    int n, m, k[16];
};
__global__ void big_args(Args a)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n) a.b[i] = a.a[i] + a.k[i & 15];
}

int main()
{
    int* d = nullptr;
    (void)hipMalloc(&d, 1 << 20);
    hipStream_t s, s2;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    hipEvent_t ev;
    (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    const int N = 20000;
    using clk = std::chrono::steady_clock;
    auto per = [&](auto fn) {
        for (int i = 0; i < 200; ++i) fn();
        (void)hipDeviceSynchronize();
        auto t0 = clk::now();
        for (int i = 0; i < N; ++i) fn();
        auto t1 = clk::now();
        (void)hipDeviceSynchronize();
        return std::chrono::duration<double, std::micro>(t1 - t0).count() / N;
    };
    Args A{d, d + 1024, 1024, 0, {}};
    double l1 = per([&] { hipLaunchKernelGGL(tiny, dim3(4), dim3(256), 0, s, d, 1024); });
    double l2 = per([&] { hipLaunchKernelGGL(big_args, dim3(4), dim3(256), 0, s, A); });
    double l3 = per([&] { hipLaunchKernelGGL(tiny, dim3(2000), dim3(256), 0, s, d, 1024); });
    double er = per([&] { (void)hipEventRecord(ev, s); });
    double we = per([&] { (void)hipStreamWaitEvent(s2, ev, 0); });
    double eq = per([&] { (void)hipEventQuery(ev); });
    std::printf("{\"launch_tiny_us\": %.3f, \"launch_big_args_us\": %.3f, \"launch_2000_blocks_us\": %.3f, "
                "\"event_record_us\": %.3f, \"stream_wait_event_us\": %.3f, \"event_query_us\": %.3f, \"calls\": %d}\n",
                l1, l2, l3, er, we, eq, N);
    return 0;
}
