// Instruction-latency floors on gfx950 for the PKO EM chain (diagnostic; not part of the product).
//   hipcc --offload-arch=gfx950 -O3 -o scripts/lat_bench scripts/lat_bench.hip && scripts/lat_bench
// One workgroup; wave 0 (and, for the barrier test, waves 1-2) run a chain of N dependent instructions between two
// s_memtime stamps.  Prints cycles per chain step.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cmath>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

#define R8(s) s s s s s s s s
#define R64(s) R8(R8(s))

constexpr int kTests = 24;

template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(static_cast<uint32_t>(u)), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(static_cast<uint32_t>(u >> 32)), CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo));
}
__device__ __forceinline__ void pl32(double& a, double& b) {
    const auto lo = __builtin_amdgcn_permlane32_swap(static_cast<unsigned>(__double2loint(a)), static_cast<unsigned>(__double2loint(b)), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(static_cast<unsigned>(__double2hiint(a)), static_cast<unsigned>(__double2hiint(b)), false, false);
    a = __hiloint2double(static_cast<int>(hi[0]), static_cast<int>(lo[0]));
    b = __hiloint2double(static_cast<int>(hi[1]), static_cast<int>(lo[1]));
}
__device__ __forceinline__ double readlane64(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}


__device__ __forceinline__ double exp_nonpos(double y) {
    const double n = rint(y * 0x1.71547652b82fep+0);
    double r = fma(-n, 0x1.62e42fefa39efp-1, y);
    r = fma(-n, 0x1.abc9e3b39803fp-56, r);
    const double r2 = r * r;
    const double a0 = 1.0 + r;
    const double a1 = fma(0x1.5555555555555p-3, r, 0.5);
    const double a2 = fma(0x1.1111111111111p-7, r, 0x1.5555555555555p-5);
    const double a3 = fma(0x1.a01a01a01a01ap-13, r, 0x1.6c16c16c16c17p-10);
    const double a4 = fma(0x1.71de3a556c734p-19, r, 0x1.a01a01a01a01ap-16);
    const double a5 = fma(0x1.ae64567f544e4p-26, r, 0x1.27e4fb7789f5cp-22);
    const double r4 = r2 * r2;
    const double b0 = fma(a1, r2, a0), b1 = fma(a3, r2, a2), b2 = fma(a5, r2, a4);
    const double r8 = r4 * r4;
    const double c0 = fma(b1, r4, b0), c1 = fma(0x1.1eed8eff8d898p-29, r4, b2);
    return ldexp(fma(c1, r8, c0), static_cast<int>(n));
}

template <int CTRL>
__device__ __forceinline__ double dpp64m(double v) {     // mov_dpp: no old operand
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(static_cast<uint32_t>(u)), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(static_cast<uint32_t>(u >> 32)), CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo));
}
__device__ __forceinline__ void pl16(double& a, double& b) {
    const auto lo = __builtin_amdgcn_permlane16_swap(static_cast<unsigned>(__double2loint(a)), static_cast<unsigned>(__double2loint(b)), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(static_cast<unsigned>(__double2hiint(a)), static_cast<unsigned>(__double2hiint(b)), false, false);
    a = __hiloint2double(static_cast<int>(hi[0]), static_cast<int>(lo[0]));
    b = __hiloint2double(static_cast<int>(hi[1]), static_cast<int>(lo[1]));
}
template <bool MOV>
__device__ __forceinline__ void totals4(double (&v)[3]) {
    double u[4] = {v[0], v[1], v[2], 0.0};
    for (int q = 0; q < 2; ++q) { pl32(u[q], u[q + 2]); u[q] += u[q + 2]; }
    pl16(u[0], u[1]);
    double t = u[0] + u[1];
    if (MOV) {
        t += dpp64m<0x128>(t); t += dpp64m<0xB1>(t); t += dpp64m<0x4E>(t); t += dpp64m<0x141>(t);
    } else {
        t += dpp64<0x128>(t); t += dpp64<0xB1>(t); t += dpp64<0x4E>(t); t += dpp64<0x141>(t);
    }
    for (int q = 0; q < 3; ++q) v[q] = readlane64(t, 16 * q);
}

__global__ void k_red(double* out, unsigned long long* cyc, double seed) {
    const int lane = threadIdx.x & 63;
    double v[3] = {seed + lane, seed * 2 - lane, seed * 0.5 + lane};
    unsigned long long t[3];
    for (int pass = 0; pass < 2; ++pass) {
        __builtin_amdgcn_s_waitcnt(0);
        t[0] = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < 32; ++r) { totals4<false>(v); v[0] += lane; asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2])); }
        __builtin_amdgcn_s_waitcnt(0);
        t[1] = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < 32; ++r) { totals4<true>(v); v[0] += lane; asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2])); }
        __builtin_amdgcn_s_waitcnt(0);
        t[2] = __builtin_amdgcn_s_memtime();
    }
    if (threadIdx.x == 0) { cyc[0] = t[1] - t[0]; cyc[1] = t[2] - t[1]; }
    out[threadIdx.x] = v[0] + v[1] + v[2];
}

__global__ void k_exp(double* out, unsigned long long* cyc, double seed) {
    const int lane = threadIdx.x & 63;
    double x = -0.001 * lane - seed * 1e-3, y = x - 0.5, z = x - 0.25, w = x - 0.125;
    unsigned long long t[4];
    for (int pass = 0; pass < 2; ++pass) {
        __builtin_amdgcn_s_waitcnt(0);
        t[0] = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < 32; ++r) { x = -exp_nonpos(x); asm volatile("" : "+v"(x)); }
        __builtin_amdgcn_s_waitcnt(0);
        t[1] = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < 32; ++r) { x = -exp_nonpos(x); y = -exp_nonpos(y); asm volatile("" : "+v"(x), "+v"(y)); }
        __builtin_amdgcn_s_waitcnt(0);
        t[2] = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < 32; ++r) { x = -exp_nonpos(x); y = -exp_nonpos(y); z = -exp_nonpos(z); w = -exp_nonpos(w); asm volatile("" : "+v"(x), "+v"(y), "+v"(z), "+v"(w)); }
        __builtin_amdgcn_s_waitcnt(0);
        t[3] = __builtin_amdgcn_s_memtime();
    }
    if (threadIdx.x == 0) { cyc[0] = t[1] - t[0]; cyc[1] = t[2] - t[1]; cyc[2] = t[3] - t[2]; }
    out[threadIdx.x] = x + y + z + w;
}

__global__ void k_lat(double* out, unsigned long long* cyc, double seed) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double x = seed + lane, y = seed * 0.5 + lane, z = seed * 0.25, w = seed * 0.125, a = 1.0000001, b = 1e-9;
    unsigned long long t[kTests + 1];
    __shared__ double sh[4 * 64];
    for (int pass = 0; pass < 2; ++pass) {     // pass 0 warms the instruction cache
    int k = 0;
#define STAMP() do { __builtin_amdgcn_s_waitcnt(0); t[k++] = __builtin_amdgcn_s_memtime(); } while (0)
    STAMP();
    // 0: 64 dependent v_fma_f64
    R64(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));)
    STAMP();
    // 1: 2 interleaved chains x 64
    R64(asm volatile("v_fma_f64 %0, %0, %2, %3\n v_fma_f64 %1, %1, %2, %3" : "+v"(x), "+v"(y) : "v"(a), "v"(b));)
    STAMP();
    // 2: 4 interleaved chains x 64
    R64(asm volatile("v_fma_f64 %0, %0, %4, %5\n v_fma_f64 %1, %1, %4, %5\n v_fma_f64 %2, %2, %4, %5\n v_fma_f64 %3, %3, %4, %5"
                     : "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(a), "v"(b));)
    STAMP();
    // 3: 64 x (dpp64 move + dependent add): the butterfly step
    asm volatile("v_mov_b32 v8, %0\n v_mov_b32 v9, %1" :: "v"(__double2loint(x)), "v"(__double2hiint(x)) : "v8", "v9");
    R64(asm volatile("v_mov_b32_dpp v10, v8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp v11, v9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_add_f64 v[8:9], v[8:9], v[10:11]" ::: "v8", "v9", "v10", "v11");)
    STAMP();
    // 4: 64 x (permlane32_swap of both halves + add)
    R64(asm volatile("v_permlane32_swap_b32 v8, v10\n v_permlane32_swap_b32 v9, v11\n v_add_f64 v[8:9], v[8:9], v[10:11]" ::: "v8", "v9", "v10", "v11");)
    STAMP();
    // 5: 64 dependent v_rcp_f64
    R64(asm volatile("v_rcp_f64 %0, %0" : "+v"(z));)
    STAMP();
    // 6: 64 x (v_readlane x2 -> s pair, v_add_f64 with the s operand)
    R64(asm volatile("v_readlane_b32 s40, v8, 5\n v_readlane_b32 s41, v9, 5\n v_add_f64 v[8:9], v[8:9], s[40:41]" ::: "v8", "v9", "s40", "s41");)
    STAMP();
    // 7: 64 dependent v_mul_f64
    R64(asm volatile("v_mul_f64 %0, %0, %1" : "+v"(w) : "v"(a));)
    STAMP();
    // 8: 64 x ds_write_b64 + ds_read_b64 round trip (same wave, no barrier)
    {
        double* p = sh + lane;
        R64(asm volatile("ds_write_b64 %1, %0\n s_waitcnt lgkmcnt(0)\n ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)"
                         : "+v"(x) : "v"(static_cast<unsigned>(reinterpret_cast<uintptr_t>(p))) : "memory");)
    }
    STAMP();
    // 9: 64 x (ds_write, barrier, ds_read) with all 3 waves of the workgroup
    {
        double* p = sh + 64 * (wid & 3) + lane;
        for (int r = 0; r < 64; ++r) {
            asm volatile("ds_write_b64 %0, %1" :: "v"(static_cast<unsigned>(reinterpret_cast<uintptr_t>(p))), "v"(x) : "memory");
            __syncthreads();
            x += sh[64 * ((wid + 1) % 3) + lane];
        }
    }
    STAMP();
    // 10: 64 x v_rndne_f64 + v_ldexp chain (exp building blocks)
    {
        int e = 1;
        R64(asm volatile("v_rndne_f64 %0, %0\n v_ldexp_f64 %0, %0, %1" : "+v"(w) : "v"(e));)
    }
    STAMP();
    // 11: 64 x 8 independent fma (issue throughput of fp64 FMA)
    {
        double q0 = x, q1 = y, q2 = z, q3 = w, q4 = x + 1, q5 = y + 1, q6 = z + 1, q7 = w + 1;
        R64(asm volatile("v_fma_f64 %0, %0, %8, %9\n v_fma_f64 %1, %1, %8, %9\n v_fma_f64 %2, %2, %8, %9\n v_fma_f64 %3, %3, %8, %9\n"
                         " v_fma_f64 %4, %4, %8, %9\n v_fma_f64 %5, %5, %8, %9\n v_fma_f64 %6, %6, %8, %9\n v_fma_f64 %7, %7, %8, %9"
                         : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(q4), "+v"(q5), "+v"(q6), "+v"(q7) : "v"(a), "v"(b));)
        x += q0 + q1 + q2 + q3 + q4 + q5 + q6 + q7;
    }
    STAMP();
    // 12: 64 dependent v_fma_f32
    {
        float f = static_cast<float>(x), fa = 1.0000001f, fb = 1e-9f;
        R64(asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f) : "v"(fa), "v"(fb));)
        x += f;
    }
    STAMP();
    // 13: 64 x dpp row_ror:8 + add (f64)
    R64(asm volatile("v_mov_b32_dpp v10, v8 row_ror:8 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp v11, v9 row_ror:8 row_mask:0xf bank_mask:0xf\n v_add_f64 v[8:9], v[8:9], v[10:11]" ::: "v8", "v9", "v10", "v11");)
    STAMP();
    // 14: 64 x ds_swizzle / ds_bpermute round trip (cross-lane via LDS crossbar)
    {
        int v = static_cast<int>(x);
        const int addr = ((lane ^ 1) << 2);
        R64(asm volatile("ds_bpermute_b32 %0, %1, %0\n s_waitcnt lgkmcnt(0)" : "+v"(v) : "v"(addr));)
        x += v;
    }
    STAMP();
    // 15: 64 x v_cmp + v_cndmask pair chain (select)
    R64(asm volatile("v_cmp_gt_f64 vcc, v[8:9], v[10:11]\n v_cndmask_b32 v8, v10, v8, vcc\n v_cndmask_b32 v9, v11, v9, vcc" ::: "v8", "v9", "vcc");)
    STAMP();

    // 16: rsq_f64 dep
    R64(asm volatile("v_rsq_f64 %0, %0" : "+v"(z));)
    STAMP();
    // 17: rcp_f32 dep
    { float f = 1.5f + lane; R64(asm volatile("v_rcp_f32 %0, %0" : "+v"(f));) x += f; }
    STAMP();
    // 18: cvt f64->f32->f64 pair
    { float f; R64(asm volatile("v_cvt_f32_f64 %1, %0\n v_cvt_f64_f32 %0, %1" : "+v"(w), "=&v"(f));) }
    STAMP();
    // 19: frexp_mant_f64 dep
    R64(asm volatile("v_frexp_mant_f64 %0, %0" : "+v"(y));)
    STAMP();
    // 20: 4 independent rcp_f64 interleaved
    { double r0 = x + 1, r1 = x + 2, r2 = x + 3, r3 = x + 4;
      R64(asm volatile("v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3" : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3));)
      x += r0 + r1 + r2 + r3; }
    STAMP();
    // 21: rsq_f32 dep
    { float f = 1.5f + lane; R64(asm volatile("v_rsq_f32 %0, %0" : "+v"(f));) x += f; }
    STAMP();
    // 22: exp_f32 dep
    { float f = 0.5f; R64(asm volatile("v_exp_f32 %0, %0" : "+v"(f));) x += f; }
    STAMP();
    // 23: add_f64 dep with readfirstlane-free s operand (s_mov constant)
    R64(asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "s"(b));)
    STAMP();
    }
    if (wid == 0 && lane == 0)
        for (int i = 0; i < kTests; ++i) cyc[i] = t[i + 1] - t[i];
    out[threadIdx.x] = x + y + z + w;
}

// accuracy of the hardware fp64 reciprocal / rsqrt seeds (max relative error over a sweep of mantissas/exponents)
__global__ void k_acc(double* err) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    double e_rcp = 0.0, e_rsq = 0.0;
    for (int k = 0; k < 64; ++k) {
        const unsigned long long bits = 0x3ff0000000000000ull + ((static_cast<unsigned long long>(i) * 64 + k) * 0x9E3779B97F4Aull & 0xfffffffffffffull);
        double x = __longlong_as_double(static_cast<long long>(bits));
        x = ldexp(x, (i % 41) - 20);
        const double r = __builtin_amdgcn_rcp(x);
        const double q = __builtin_amdgcn_rsq(x);
        const double er = fabs(r * x - 1.0);
        const double eq = fabs(q * q * x - 1.0);
        e_rcp = er > e_rcp ? er : e_rcp;
        e_rsq = eq > e_rsq ? eq : e_rsq;
    }
    err[2 * i] = e_rcp;
    err[2 * i + 1] = e_rsq;
}

int main() {
    {
        const int n = 1 << 16;
        double* d;
        CK(hipMalloc(&d, 2 * n * sizeof(double)));
        hipLaunchKernelGGL(k_acc, dim3(n / 256), dim3(256), 0, 0, d);
        CK(hipDeviceSynchronize());
        double* h = new double[2 * n];
        CK(hipMemcpy(h, d, 2 * n * sizeof(double), hipMemcpyDeviceToHost));
        double mr = 0, mq = 0;
        for (int i = 0; i < n; ++i) { mr = h[2 * i] > mr ? h[2 * i] : mr; mq = h[2 * i + 1] > mq ? h[2 * i + 1] : mq; }
        std::printf("v_rcp_f64 max rel err %.3e (2^%.1f), v_rsq_f64 (x q^2 - 1) %.3e (2^%.1f)\n", mr, std::log2(mr), mq, std::log2(mq));
        delete[] h;
    }
    double* d_out;
    unsigned long long* d_cyc;
    CK(hipMalloc(&d_out, 256 * sizeof(double)));
    CK(hipMalloc(&d_cyc, kTests * sizeof(unsigned long long)));
    const char* names[kTests] = {"fma_f64 dep",       "fma_f64 2 chains", "fma_f64 4 chains",  "dpp64 quad + add",
                                 "permlane32 + add",  "rcp_f64 dep",      "readlane + s add",  "mul_f64 dep",
                                 "ds write+read",     "ds+barrier(3w)",   "rndne+ldexp",       "fma_f64 8 indep",
                                 "fma_f32 dep",       "dpp64 ror8 + add", "bpermute",          "cmp+cndmask64",
                                 "rsq_f64 dep", "rcp_f32 dep", "cvt f64>f32>f64", "frexp_mant dep", "rcp_f64 4 indep", "rsq_f32 dep",
                                 "exp_f32 dep", "add_f64 s-op dep"};
    {
        for (int rep = 0; rep < 2; ++rep) { hipLaunchKernelGGL(k_exp, dim3(1), dim3(64), 0, 0, d_out, d_cyc, 1.0); CK(hipDeviceSynchronize()); }
        unsigned long long h[3];
        CK(hipMemcpy(h, d_cyc, sizeof(h), hipMemcpyDeviceToHost));
        std::printf("exp_nonpos chain: 1x %.1f, 2x %.1f, 4x %.1f cycles per iteration (32 iterations)\n", h[0] / 32.0, h[1] / 32.0, h[2] / 32.0);
    }
    {
        for (int rep = 0; rep < 2; ++rep) { hipLaunchKernelGGL(k_red, dim3(1), dim3(64), 0, 0, d_out, d_cyc, 1.0); CK(hipDeviceSynchronize()); }
        unsigned long long h[2];
        CK(hipMemcpy(h, d_cyc, sizeof(h), hipMemcpyDeviceToHost));
        std::printf("wave_totals4<3>: update_dpp %.1f, mov_dpp %.1f cycles per reduction\n", h[0] / 32.0, h[1] / 32.0);
    }
    for (int waves = 1; waves <= 3; waves += 2) {
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k_lat, dim3(1), dim3(64 * waves), 0, 0, d_out, d_cyc, 1.0 + rep);
            CK(hipDeviceSynchronize());
        }
        unsigned long long h[kTests];
        CK(hipMemcpy(h, d_cyc, sizeof(h), hipMemcpyDeviceToHost));
        std::printf("waves=%d\n", waves);
        for (int i = 0; i < kTests; ++i) std::printf("  %-20s %7.2f cycles / step (64 steps: %llu)\n", names[i], h[i] / 64.0, h[i]);
    }
    return 0;
}
