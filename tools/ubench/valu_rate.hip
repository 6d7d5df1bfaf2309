// Microbenchmark: VALU issue cost of single instructions on gfx950 at 4 waves per SIMD
// (the megakernel's occupancy).  Each lane runs 8 independent dependency chains of one
// instruction (inline asm, so exactly that instruction); the kernel time over
// (waves x N x 8) gives cycles per wave-instruction per SIMD at the reported clock.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/valu_rate.hip -o tools/ubench/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN8(ASM, ...)                                        \
    _Pragma("unroll") for (int i = 0; i < 8; i++) asm volatile(ASM : __VA_ARGS__);

template <int KIND>
__global__ __launch_bounds__(1024) void k(float* outf, int n) {
    float f[8];
    double d[8];
    unsigned u[8];
    for (int i = 0; i < 8; i++) {
        f[i] = threadIdx.x * 1e-3f + i;
        d[i] = threadIdx.x * 1e-3 + i;
        u[i] = threadIdx.x + i;
    }
    const float a = 0.999f, b = 1.0f;
    const double da = 0.999, db = 1.0;
#pragma unroll 1
    for (int it = 0; it < n; it++) {
        if (KIND == 0) CHAIN8("v_fma_f32 %0, %0, %1, %2", "+v"(f[i]) : "v"(a), "v"(b))
        if (KIND == 1) CHAIN8("v_fma_f64 %0, %0, %1, %2", "+v"(d[i]) : "v"(da), "v"(db))
        if (KIND == 2) CHAIN8("v_mul_f64 %0, %0, %1", "+v"(d[i]) : "v"(da))
        if (KIND == 3) CHAIN8("v_max3_f32 %0, %0, %1, %2", "+v"(f[i]) : "v"(a), "v"(b))
        if (KIND == 4) CHAIN8("v_min_f32 %0, %0, %1", "+v"(f[i]) : "v"(a))
        if (KIND == 5) CHAIN8("v_max_f64 %0, %0, %1", "+v"(d[i]) : "v"(da))
        if (KIND == 6) CHAIN8("v_add_u32 %0, %0, %1", "+v"(u[i]) : "v"(u[0]))
        if (KIND == 7) CHAIN8("v_mul_lo_u32 %0, %0, %1", "+v"(u[i]) : "v"(u[0]))
        if (KIND == 8) CHAIN8("v_cndmask_b32 %0, %0, %1, vcc", "+v"(u[i]) : "v"(u[0]) : "vcc")
        if (KIND == 9) CHAIN8("v_pk_fma_f32 %0, %0, %1, %2", "+v"(d[i]) : "v"(da), "v"(db))
        if (KIND == 10) CHAIN8("v_add_f64 %0, %0, %1", "+v"(d[i]) : "v"(da))
        if (KIND == 11) CHAIN8("v_lshl_add_u64 %0, %0, 1, %1", "+v"(d[i]) : "v"(db))
    }
    float s = 0;
    for (int i = 0; i < 8; i++) s += f[i] + (float)u[i] + (float)d[i];
    outf[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    const int blocks = cus, threads = 1024, n = 20000;  // 16 waves/CU = 4 per SIMD
    float* of;
    hipMalloc(&of, blocks * threads * 4);
    const char* names[] = {"v_fma_f32",     "v_fma_f64", "v_mul_f64",    "v_max3_f32",
                           "v_min_f32",     "v_max_f64", "v_add_u32",    "v_mul_lo_u32",
                           "v_cndmask_b32", "v_pk_fma_f32", "v_add_f64", "v_lshl_add_u64"};
    void (*ks[])(float*, int) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>, k<9>, k<10>, k<11>};
    for (int t = 0; t < 12; t++) {
        hipLaunchKernelGGL(ks[t], dim3(blocks), dim3(threads), 0, 0, of, 100);
        hipDeviceSynchronize();
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(ks[t], dim3(blocks), dim3(threads), 0, 0, of, n);
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
