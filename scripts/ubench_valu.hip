// Throughput of the VALU instructions the check node uses, on gfx950.
// Each thread runs 8 independent chains of one instruction (inline asm, so
// nothing folds); the grid fills every SIMD with W waves. Reports cycles per
// wave-instruction per SIMD (clock from the -c argument, default 2.4 GHz is
// NOT assumed: s_memtime is read inside the kernel).
//   hipcc --offload-arch=gfx950 -O3 -o ab/ubench_valu scripts/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define ITER 2048

#define BODY8(INS)                                                                         \
    asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS        \
                     " %3, %3, %8\n\t" INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS         \
                     " %6, %6, %8\n\t" INS " %7, %7, %8"                                      \
                 : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) \
                 : "v"(s))

template <int OP>
__global__ __launch_bounds__(256) void k_bench(unsigned long long *cyc, double *sink, double seed)
{
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (OP < 4) {
        double r0 = seed + threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5,
               r6 = r0 + 6, r7 = r0 + 7, s = seed * 0.5;
        for (int i = 0; i < ITER; ++i) {
            if constexpr (OP == 0) BODY8("v_add_f64");
            if constexpr (OP == 1) BODY8("v_min_f64");
            if constexpr (OP == 2) BODY8("v_mul_f64");
            if constexpr (OP == 3) BODY8("v_max_f64");
        }
        sink[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
    } else {
        float r0 = seed + threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5,
              r6 = r0 + 6, r7 = r0 + 7, s = seed * 0.5;
        for (int i = 0; i < ITER; ++i) {
            if constexpr (OP == 4) BODY8("v_add_f32");
            if constexpr (OP == 5) BODY8("v_min_f32");
            if constexpr (OP == 6) BODY8("v_xor_b32");
            if constexpr (OP == 7) BODY8("v_sub_u32");
        }
        sink[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// v_cmp_*_f64 / u64 throughput: 8 independent compares per step, results ORed
// into SGPR pairs is awkward in asm; use VOP3 form writing an SGPR pair.
template <int OP>
__global__ __launch_bounds__(256) void k_cmp(unsigned long long *cyc, double *sink, double seed)
{
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    double a = seed + threadIdx.x, b = seed * 0.5;
    unsigned long long m = 0;
    for (int i = 0; i < ITER; ++i) {
        unsigned long long c0, c1, c2, c3, c4, c5, c6, c7;
#define CMP8(INS, A)                                                                                   \
    asm volatile(INS " %0, " A ", %9\n\t" INS " %1, " A ", %9\n\t" INS " %2, " A ", %9\n\t" INS " %3, " A        \
                 ", %9\n\t" INS " %4, " A ", %9\n\t" INS " %5, " A ", %9\n\t" INS " %6, " A ", %9\n\t" INS " %7, " A \
                 ", %9"                                                                                       \
                 : "=s"(c0), "=s"(c1), "=s"(c2), "=s"(c3), "=s"(c4), "=s"(c5), "=s"(c6), "=s"(c7)            \
                 : "v"(a), "v"(b))
        if constexpr (OP == 0) CMP8("v_cmp_le_f64_e64", "%8");
        if constexpr (OP == 1) CMP8("v_cmp_le_u64_e64", "%8");
        if constexpr (OP == 2) CMP8("v_cmp_eq_f64_e64", "|%8|");   // the check node's argmin mask
        if constexpr (OP == 3) CMP8("v_cmp_eq_u64_e64", "%8");
        m ^= c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = (double)m;
}

template <typename K>
static void run(const char *name, K kern, int waves_per_simd)
{
    int cus = 256;
    int blocks = cus * waves_per_simd;   // 256-thread block = 4 waves = one per SIMD
    unsigned long long *cyc;
    double *sink;
    hipMalloc(&cyc, blocks * 8);
    hipMalloc(&sink, (size_t)blocks * 256 * 8);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, cyc, sink, 1.0);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, cyc, sink, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long *h = (unsigned long long *)malloc(blocks * 8);
    hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < blocks; ++i) avg += (double)h[i];
    avg /= blocks;
    // per SIMD: waves_per_simd waves x ITER x 8 instructions
    const double ins = (double)waves_per_simd * ITER * 8;
    // s_memtime counts at the shader clock; cycles per instruction per SIMD
    printf("%-14s W=%d  %.2f memtime-cyc/instr/SIMD   wall %.3f ms -> %.2f ns/instr/SIMD\n", name, waves_per_simd,
           avg / ins * waves_per_simd / waves_per_simd, ms, ms * 1e6 / ins);
    free(h);
    hipFree(cyc);
    hipFree(sink);
}

int main()
{
    for (int w : {1, 4, 8}) {
        run("v_add_f64", k_bench<0>, w);
        run("v_min_f64", k_bench<1>, w);
        run("v_mul_f64", k_bench<2>, w);
        run("v_max_f64", k_bench<3>, w);
        run("v_add_f32", k_bench<4>, w);
        run("v_min_f32", k_bench<5>, w);
        run("v_xor_b32", k_bench<6>, w);
        run("v_sub_u32", k_bench<7>, w);
        run("v_cmp_le_f64", k_cmp<0>, w);
        run("v_cmp_le_u64", k_cmp<1>, w);
        run("v_cmp_eq_f64|a|", k_cmp<2>, w);
        run("v_cmp_eq_u64", k_cmp<3>, w);
    }
    return 0;
}
