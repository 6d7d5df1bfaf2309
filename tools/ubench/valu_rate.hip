// Microbenchmark: VALU issue rate of f32 / f64 / int ops on gfx950 with 4 waves per SIMD
// (the megakernel's occupancy).  Each lane runs 8 independent dependency chains of N ops;
// the kernel's time over (waves x N x 8) gives cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>

template <int KIND>
__global__ __launch_bounds__(1024) void k(float* outf, double* outd, int n, float sf, double sd) {
    float f[8];
    double d[8];
    unsigned u[8];
    for (int i = 0; i < 8; i++) {
        f[i] = threadIdx.x * 1e-3f + i;
        d[i] = threadIdx.x * 1e-3 + i;
        u[i] = threadIdx.x + i;
    }
#pragma unroll 1
    for (int it = 0; it < n; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (KIND == 0) f[i] = __builtin_fmaf(f[i], sf, 1.0f);
            if (KIND == 1) d[i] = __builtin_fma(d[i], sd, 1.0);
            if (KIND == 2) d[i] = d[i] * sd;
            if (KIND == 3) u[i] = u[i] * 2654435761u + 1u;  // v_mad_u32_u24? no: v_mul_lo_u32
            if (KIND == 4) f[i] = __builtin_fminf(f[i], sf);
            if (KIND == 5) d[i] = __builtin_fmin(d[i], sd);
            if (KIND == 6) u[i] = u[i] + 0x9e3779b9u;
        }
    }
    float a = 0; double b = 0;
    for (int i = 0; i < 8; i++) { a += f[i] + (float)u[i]; b += d[i]; }
    outf[blockIdx.x * blockDim.x + threadIdx.x] = a;
    outd[blockIdx.x * blockDim.x + threadIdx.x] = b;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    const int blocks = cus, threads = 1024, n = 20000;  // 16 waves/CU = 4 per SIMD
    float* of; double* od;
    hipMalloc(&of, blocks * threads * 4);
    hipMalloc(&od, blocks * threads * 8);
    const char* names[] = {"v_fma_f32", "v_fma_f64", "v_mul_f64", "v_mul_lo_u32", "v_min_f32", "v_min_f64", "v_add_u32"};
    void (*ks[])(float*, double*, int, float, double) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>};
    for (int t = 0; t < 7; t++) {
        hipLaunchKernelGGL(ks[t], dim3(blocks), dim3(threads), 0, 0, of, od, 100, 0.999f, 0.999);
        hipDeviceSynchronize();
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(ks[t], dim3(blocks), dim3(threads), 0, 0, of, od, n, 0.999f, 0.999);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double simd_instr = (double)blocks * (threads / 64) * n * 8 / (cus * 4);  // wave-instr per SIMD
        const double cycles = ms * 1e-3 * clk * 1e3;  // at the reported clock
        printf("%-14s %8.3f ms  %.2f cycles per wave-instruction per SIMD (at %d MHz)\n", names[t], ms,
               cycles / simd_instr, clk / 1000);
    }
    return 0;
}
