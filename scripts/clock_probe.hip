// Shader clock under load: s_memtime (core clock) against s_memrealtime
// (100 MHz constant), per workgroup over a VALU-bound loop on every CU.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned long long *out, int iters)
{
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    double a = threadIdx.x * 1e-3, b = 1.0000001;
    for (int i = 0; i < iters; ++i) { a = a * b + 1e-9; b = b * a - 1e-9; }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { out[2 * blockIdx.x] = t1 - t0; out[2 * blockIdx.x + 1] = r1 - r0; }
    if (a == 12345.0) out[0] = 0;
}
int main()
{
    unsigned long long *d, h[2 * 2048];
    hipMalloc(&d, sizeof h);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k, dim3(2048), dim3(512), 0, 0, d, 200000);
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        double st = 0, sr = 0;
        for (int i = 0; i < 2048; ++i) { st += h[2 * i]; sr += h[2 * i + 1]; }
        printf("rep %d: memtime/memrealtime = %.1f -> clock %.3f GHz (realtime 100 MHz)\n", rep, st / sr, st / sr * 0.1);
    }
    return 0;
}
