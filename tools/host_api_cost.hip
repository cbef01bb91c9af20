// host_api_cost.hip — host-side cost of the HIP calls the TBD loop makes per
// frame (event record, stream wait, empty kernel launch, event query), each
// timed over 2000 calls on the GPU box.
// Build: hipcc --offload-arch=gfx950 -O2 tools/host_api_cost.hip -o tools/bin/host_api_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void empty_kernel(int* p) { if (p && threadIdx.x == 1000) p[0] = 1; }

int main()
{
    using clk = std::chrono::steady_clock;
    hipStream_t a, b;
    hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
    hipEvent_t ev, evt;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    hipEventCreate(&evt);
    const int N = 2000;
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, a, nullptr);
    hipDeviceSynchronize();
    auto t0 = clk::now();
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(empty_kernel, dim3(64), dim3(64), 0, a, nullptr);
    auto t1 = clk::now();
    hipDeviceSynchronize();
    auto t2 = clk::now();
    for (int i = 0; i < N; ++i) hipEventRecord(ev, a);
    auto t3 = clk::now();
    for (int i = 0; i < N; ++i) hipEventRecord(evt, a);
    auto t4 = clk::now();
    for (int i = 0; i < N; ++i) hipStreamWaitEvent(b, ev, 0);
    auto t5 = clk::now();
    hipDeviceSynchronize();
    auto t6 = clk::now();
    for (int i = 0; i < N; ++i) (void)hipEventQuery(ev);
    auto t7 = clk::now();
    auto us = [&](clk::time_point x, clk::time_point y) { return std::chrono::duration<double, std::micro>(y - x).count() / N; };
    printf("launch %.2f us, event record (no timing) %.2f us, event record (timing) %.2f us, stream wait %.2f us, "
           "event query %.2f us\n", us(t0, t1), us(t2, t3), us(t3, t4), us(t4, t5), us(t6, t7));
    return 0;
}
