// Microbenchmark: VALU issue cost per wave-instruction per SIMD on gfx950, by instruction
// class, at 4 and 8 waves per SIMD (price the roofline from measured costs).
//
// Each lane runs 8 independent dependency chains of one instruction written in inline asm
// (exactly that instruction), every source operand but the chain register an SGPR or an
// inline constant (no VGPR bank conflicts).  The kernel runs long enough (~10-40 ms) for
// the chip to settle its clock, and the clock is measured inside the kernel: each wave
// stamps s_memtime (shader clock) and s_memrealtime (100 MHz) around its loop, so
//   cycles per wave-instruction per SIMD = (shader cycles of the loop) x SIMDs_used
//                                           / (wave-instructions issued on the chip)
// is independent of DVFS.  (MI355X_MICROARCH.md: a wave64 32-bit VALU op issues over 2
// cycles on a SIMD-32; one wave alone sustains 4.)
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/valu_rate.hip -o tools/ubench/valu_rate
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

// 8 rounds of the 8 chains per loop iteration: 64 instructions per taken branch
#define CHAIN8(ASM, ...) \
    _Pragma("unroll") for (int r = 0; r < 8; r++) _Pragma("unroll") for (int i = 0; i < 8; i++) asm volatile(ASM : __VA_ARGS__);

struct Stamp {
    unsigned long long t0, t1, r0, r1;
    unsigned hw, xcc, pad0, pad1;
};

template <int KIND>
__global__ __launch_bounds__(256) void k(float* outf, Stamp* st, int n, unsigned sa) {
    float f[8];
    double d[8];
    unsigned u[8];
    for (int i = 0; i < 8; i++) {
        f[i] = threadIdx.x * 1e-3f + i;
        d[i] = threadIdx.x * 1e-3 + i;
        u[i] = threadIdx.x + i;
    }
    // wave-uniform operands: compiled into SGPRs ("s" constraint)
    const float fs = __builtin_amdgcn_readfirstlane(__float_as_uint(0.999f)) ? 0.999f : 1.0f;
    const unsigned us = __builtin_amdgcn_readfirstlane(sa);
    const double ds = (double)fs;
    // per-lane (VGPR) operands
    const float fv = 0.999f + threadIdx.x * 1e-9f, fw = 1.0f - threadIdx.x * 1e-9f;
    const double dv = fv, dw = fw;
    const unsigned uv = threadIdx.x * 3u + 1u;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll 1
    for (int it = 0; it < n; it++) {
        if (KIND == 0) CHAIN8("v_fma_f32 %0, %0, %1, 1.0", "+v"(f[i]) : "s"(fs))
        if (KIND == 1) CHAIN8("v_pk_fma_f32 %0, %0, %1, %0", "+v"(d[i]) : "s"(ds))
        if (KIND == 2) CHAIN8("v_add_f32 %0, %0, %1", "+v"(f[i]) : "s"(fs))
        if (KIND == 3) CHAIN8("v_mul_f32 %0, %0, %1", "+v"(f[i]) : "s"(fs))
        if (KIND == 4) CHAIN8("v_min_f32 %0, %0, %1", "+v"(f[i]) : "s"(fs))
        if (KIND == 5) CHAIN8("v_max3_f32 %0, %0, %1, 1.0", "+v"(f[i]) : "s"(fs))
        if (KIND == 6) CHAIN8("v_fma_f64 %0, %0, %1, 1.0", "+v"(d[i]) : "s"(ds))
        if (KIND == 7) CHAIN8("v_add_f64 %0, %0, %1", "+v"(d[i]) : "s"(ds))
        if (KIND == 8) CHAIN8("v_mul_f64 %0, %0, %1", "+v"(d[i]) : "s"(ds))
        if (KIND == 9) CHAIN8("v_max_f64 %0, %0, %1", "+v"(d[i]) : "s"(ds))
        if (KIND == 10) CHAIN8("v_add_u32 %0, %0, %1", "+v"(u[i]) : "s"(us))
        if (KIND == 11) CHAIN8("v_mul_lo_u32 %0, %0, %1", "+v"(u[i]) : "s"(us))
        if (KIND == 12) CHAIN8("v_cndmask_b32 %0, %0, 1, s[0:1]", "+v"(u[i]) : : "s0", "s1")
        if (KIND == 13) CHAIN8("v_and_b32 %0, %0, %1", "+v"(u[i]) : "s"(us))
        if (KIND == 14) CHAIN8("v_lshl_add_u64 %0, %0, 1, %1", "+v"(d[i]) : "s"(ds))
        if (KIND == 15) CHAIN8("v_mad_u64_u32 %0, s[0:1], %1, %2, %0", "+v"(d[i]) : "v"(u[i]), "s"(us) : "s0", "s1")
        if (KIND == 16) CHAIN8("v_sqrt_f32 %0, %0", "+v"(f[i]) :)
        if (KIND == 17) CHAIN8("v_sqrt_f64 %0, %0", "+v"(d[i]) :)
        if (KIND == 18) CHAIN8("v_rcp_f64 %0, %0", "+v"(d[i]) :)
        if (KIND == 19) CHAIN8("v_cvt_f32_f64 %0, %1", "=v"(f[i]) : "v"(d[i]))
        if (KIND == 20) CHAIN8("v_mov_b32 %0, %1", "=v"(u[i]) : "s"(us))
        if (KIND == 21) CHAIN8("v_cmp_lt_f32 vcc, %0, %1", "+v"(f[i]) : "s"(fs) : "vcc")
        if (KIND == 22) CHAIN8("v_ldexp_f64 %0, %0, %1", "+v"(d[i]) : "s"(us))
        if (KIND == 23) CHAIN8("v_cmp_lt_f64 vcc, %0, %1", "+v"(d[i]) : "s"(ds) : "vcc")
        // all-VGPR operands, shortest encodings (VOP1 / VOP2: 4 bytes)
        if (KIND == 24) CHAIN8("v_add_f32_e32 %0, %1, %0", "+v"(f[i]) : "v"(fv))
        if (KIND == 25) CHAIN8("v_fmac_f32_e32 %0, %1, %2", "+v"(f[i]) : "v"(fv), "v"(fw))
        if (KIND == 26) CHAIN8("v_fma_f32 %0, %0, %1, %2", "+v"(f[i]) : "v"(fv), "v"(fw))
        if (KIND == 27) CHAIN8("v_pk_fma_f32 %0, %0, %1, %2", "+v"(d[i]) : "v"(dv), "v"(dw))
        if (KIND == 28) CHAIN8("v_add_u32_e32 %0, %1, %0", "+v"(u[i]) : "v"(uv))
        if (KIND == 29) CHAIN8("v_mov_b32_e32 %0, %1", "=v"(u[i]) : "v"(uv))
        if (KIND == 30) CHAIN8("v_add_f64 %0, %0, %1", "+v"(d[i]) : "v"(dv))
        if (KIND == 31) CHAIN8("v_fma_f64 %0, %0, %1, %2", "+v"(d[i]) : "v"(dv), "v"(dw))
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    float s = 0;
    for (int i = 0; i < 8; i++) s += f[i] + (float)u[i] + (float)d[i];
    outf[blockIdx.x * blockDim.x + threadIdx.x] = s;
    // HW_ID (simd, cu, sh, se) and XCC_ID name the SIMD the wave ran on
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4) & 0xFF30u;
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xFu;
    if ((threadIdx.x & 63) == 0) st[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = Stamp{t0, t1, r0, r1, hw, xcc, 0, 0};
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const char* names[] = {"v_fma_f32",     "v_pk_fma_f32", "v_add_f32",     "v_mul_f32",      "v_min_f32",
                           "v_max3_f32",    "v_fma_f64",    "v_add_f64",     "v_mul_f64",      "v_max_f64",
                           "v_add_u32",     "v_mul_lo_u32", "v_cndmask_b32", "v_and_b32",      "v_lshl_add_u64",
                           "v_mad_u64_u32", "v_sqrt_f32",   "v_sqrt_f64",    "v_rcp_f64",      "v_cvt_f32_f64",
                           "v_mov_b32",     "v_cmp_lt_f32", "v_ldexp_f64",   "v_cmp_lt_f64",
                           "v_add_f32_e32 v", "v_fmac_f32_e32 v", "v_fma_f32 v", "v_pk_fma_f32 v", "v_add_u32_e32 v",
                           "v_mov_b32_e32 v", "v_add_f64 v", "v_fma_f64 v"};
    void (*ks[])(float*, Stamp*, int, unsigned) = {k<0>,  k<1>,  k<2>,  k<3>,  k<4>,  k<5>,  k<6>,  k<7>,
                                                   k<8>,  k<9>,  k<10>, k<11>, k<12>, k<13>, k<14>, k<15>,
                                                   k<16>, k<17>, k<18>, k<19>, k<20>, k<21>, k<22>, k<23>,
                                                   k<24>, k<25>, k<26>, k<27>, k<28>, k<29>, k<30>, k<31>};
    const int nk = sizeof(ks) / sizeof(ks[0]);
    const int threads = 256;
    printf("# cycles per wave64 VALU instruction per SIMD (in-kernel shader clock; 8 independent chains per lane,\n"
           "# SGPR / inline-constant operands).  waves/SIMD = blocks per CU x 4 waves / 4 SIMDs\n");
    printf("%-16s %8s %8s %10s %10s %10s %6s %5s\n", "instruction", "w/SIMD", "cycles", "chip cyc", "clock GHz", "kernel ms",
           "SIMDs", "waves");
    for (int wps : {1, 4, 8}) {
        const int blocks = cus * wps;  // 256-thread blocks: wps blocks per CU = wps waves per SIMD
        float* of;
        Stamp* st;
        hipMalloc(&of, (size_t)blocks * threads * 4);
        hipMalloc(&st, (size_t)blocks * (threads / 64) * sizeof(Stamp));
        std::vector<Stamp> h((size_t)blocks * (threads / 64));
        for (int t = 0; t < nk; t++) {
            const int n = wps == 1 ? 5000 : 12500;
            hipLaunchKernelGGL(ks[t], dim3(blocks), dim3(threads), 0, 0, of, st, 200, 1u);  // warm
            hipDeviceSynchronize();
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(ks[t], dim3(blocks), dim3(threads), 0, 0, of, st, n, 1u);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(h.data(), st, h.size() * sizeof(Stamp), hipMemcpyDeviceToHost);
            // Per SIMD (xcc, se, sh, cu, simd): the span from its first wave's start to its last
            // wave's end, over the wave-instructions its waves issued; the median over SIMDs.
            // (The shader clock is one counter per SIMD's CU, so spans compare within a SIMD.)
            std::map<unsigned long long, std::pair<unsigned long long, unsigned long long>> span;
            std::map<unsigned long long, int> waves;
            std::vector<double> ghz;
            for (const Stamp& s : h) {
                const unsigned long long key = ((unsigned long long)s.xcc << 32) | s.hw;
                auto it = span.find(key);
                if (it == span.end()) span[key] = {s.t0, s.t1};
                else it->second = {std::min(it->second.first, s.t0), std::max(it->second.second, s.t1)};
                waves[key]++;
                ghz.push_back((double)(s.t1 - s.t0) / ((double)(s.r1 - s.r0) * 10.0));  // 100 MHz realtime
            }
            std::vector<double> per_simd, wv;
            for (auto& kv : span) {
                const int nw = waves[kv.first];
                per_simd.push_back((double)(kv.second.second - kv.second.first) / ((double)nw * n * 64));
                wv.push_back(nw);
            }
            std::sort(per_simd.begin(), per_simd.end());
            std::sort(ghz.begin(), ghz.end());
            std::sort(wv.begin(), wv.end());
            const double per = per_simd[per_simd.size() / 2], g = ghz[ghz.size() / 2];
            // the chip-wide view: every SIMD's wave-instructions over the kernel's cycles
            const double chip = ms * 1e-3 * g * 1e9 / ((double)blocks * (threads / 64) * n * 64 / (cus * 4));
            printf("%-16s %8d %8.2f %10.2f %10.3f %10.3f %6zu %5.0f\n", names[t], wps, per, chip, g, ms, span.size(), wv[wv.size() / 2]);
            hipEventDestroy(e0);
            hipEventDestroy(e1);
        }
        hipFree(of);
        hipFree(st);
    }
    return 0;
}
