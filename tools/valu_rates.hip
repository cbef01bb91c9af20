// valu_rates.hip — issue rate of the VALU instructions the PyrLK kernel is built
// from, on one MI355X: N independent chains per wave, W waves per SIMD, cycles
// per wave-instruction per SIMD from s_memtime around the loop.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rates.hip -o tools/bin/valu_rates
#include <hip/hip_runtime.h>

#include <cstdio>

#define LOOP 4096

template <int OP>
__global__ void rate_kernel(int* out, long long* cyc, int seed)
{
    int a0 = threadIdx.x + seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17,
        a7 = a0 * 19;
    const int b = seed * 0x10001;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < LOOP; ++i) {
        if constexpr (OP == 0) asm volatile("v_dot2_i32_i16 %0, %8, %8, %0\nv_dot2_i32_i16 %1, %8, %8, %1\nv_dot2_i32_i16 %2, %8, %8, %2\nv_dot2_i32_i16 %3, %8, %8, %3\nv_dot2_i32_i16 %4, %8, %8, %4\nv_dot2_i32_i16 %5, %8, %8, %5\nv_dot2_i32_i16 %6, %8, %8, %6\nv_dot2_i32_i16 %7, %8, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
        else if constexpr (OP == 1) asm volatile("v_add_u32 %0, %8, %0\nv_add_u32 %1, %8, %1\nv_add_u32 %2, %8, %2\nv_add_u32 %3, %8, %3\nv_add_u32 %4, %8, %4\nv_add_u32 %5, %8, %5\nv_add_u32 %6, %8, %6\nv_add_u32 %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
        else if constexpr (OP == 2) asm volatile("v_fma_f32 %0, %8, %8, %0\nv_fma_f32 %1, %8, %8, %1\nv_fma_f32 %2, %8, %8, %2\nv_fma_f32 %3, %8, %8, %3\nv_fma_f32 %4, %8, %8, %4\nv_fma_f32 %5, %8, %8, %5\nv_fma_f32 %6, %8, %8, %6\nv_fma_f32 %7, %8, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
        else if constexpr (OP == 3) asm volatile("v_pk_add_u16 %0, %8, %0\nv_pk_add_u16 %1, %8, %1\nv_pk_add_u16 %2, %8, %2\nv_pk_add_u16 %3, %8, %3\nv_pk_add_u16 %4, %8, %4\nv_pk_add_u16 %5, %8, %5\nv_pk_add_u16 %6, %8, %6\nv_pk_add_u16 %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
        else if constexpr (OP == 4) asm volatile("v_ashrrev_i32_sdwa %0, 9, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\nv_ashrrev_i32_sdwa %1, 9, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\nv_ashrrev_i32_sdwa %2, 9, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\nv_ashrrev_i32_sdwa %3, 9, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\nv_ashrrev_i32_sdwa %4, 9, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\nv_ashrrev_i32_sdwa %5, 9, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\nv_ashrrev_i32_sdwa %6, 9, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\nv_ashrrev_i32_sdwa %7, 9, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
        else if constexpr (OP == 5) asm volatile("v_add_u32_dpp %0, %8, %0 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %1, %8, %1 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %2, %8, %2 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %3, %8, %3 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %4, %8, %4 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %5, %8, %5 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %6, %8, %6 row_shr:1 row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %7, %8, %7 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
        else if constexpr (OP == 6) asm volatile("v_dot4_u32_u8 %0, %8, %8, %0\nv_dot4_u32_u8 %1, %8, %8, %1\nv_dot4_u32_u8 %2, %8, %8, %2\nv_dot4_u32_u8 %3, %8, %8, %3\nv_dot4_u32_u8 %4, %8, %8, %4\nv_dot4_u32_u8 %5, %8, %8, %5\nv_dot4_u32_u8 %6, %8, %8, %6\nv_dot4_u32_u8 %7, %8, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
        else if constexpr (OP == 7) asm volatile("v_dot2_u32_u16 %0, %8, %8, %0\nv_dot2_u32_u16 %1, %8, %8, %1\nv_dot2_u32_u16 %2, %8, %8, %2\nv_dot2_u32_u16 %3, %8, %8, %3\nv_dot2_u32_u16 %4, %8, %8, %4\nv_dot2_u32_u16 %5, %8, %8, %5\nv_dot2_u32_u16 %6, %8, %8, %6\nv_dot2_u32_u16 %7, %8, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
        else if constexpr (OP == 8) asm volatile("v_mad_u32_u24 %0, %8, %8, %0\nv_mad_u32_u24 %1, %8, %8, %1\nv_mad_u32_u24 %2, %8, %8, %2\nv_mad_u32_u24 %3, %8, %8, %3\nv_mad_u32_u24 %4, %8, %8, %4\nv_mad_u32_u24 %5, %8, %8, %5\nv_mad_u32_u24 %6, %8, %8, %6\nv_mad_u32_u24 %7, %8, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
static void run(const char* name, int waves_per_simd)
{
    const int cus = 256, block = 64 * 4 * waves_per_simd;  // 4 SIMDs per CU
    int* out;
    long long* cyc;
    (void)hipMalloc(&out, sizeof(int) * cus * block);
    (void)hipMalloc(&cyc, sizeof(long long) * cus);
    hipLaunchKernelGGL(rate_kernel<OP>, dim3(cus), dim3(block), 0, 0, out, cyc, 3);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(rate_kernel<OP>, dim3(cus), dim3(block), 0, 0, out, cyc, 5);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    long long c[256];
    (void)hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    long long mx = 0;
    for (int i = 0; i < cus; ++i) mx = c[i] > mx ? c[i] : mx;
    const double instr_per_simd = (double)LOOP * 8 * waves_per_simd;  // wave-instructions per SIMD
    // s_memtime ticks at the shader clock on gfx950 (guide constants table)
    // event time: wave-instructions per SIMD per ns, and cycles at 2.1 GHz (the loaded clock)
    std::printf("%-22s waves/SIMD %d: s_memtime %6.2f per wave-instr per SIMD; event %.3f ms = %.2f ns per "
                "wave-instr per SIMD (%.2f cycles at 2.1 GHz)\n", name, waves_per_simd, (double)mx / instr_per_simd,
                ms, ms * 1e6 / instr_per_simd, ms * 1e6 / instr_per_simd * 2.1);
    (void)hipFree(out);
    (void)hipFree(cyc);
}

int main()
{
    for (int w : {1, 2, 4}) {
        run<0>("v_dot2_i32_i16", w);
        run<1>("v_add_u32", w);
        run<2>("v_fma_f32", w);
        run<3>("v_pk_add_u16", w);
        run<4>("v_ashrrev sdwa", w);
        run<5>("v_add_u32 dpp", w);
        run<6>("v_dot4_u32_u8", w);
        run<7>("v_dot2_u32_u16", w);
        run<8>("v_mad_u32_u24", w);
    }
    return 0;
}
