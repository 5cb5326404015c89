// lo_pko_body.h — PKO adaptive Huber scale (AdaptiveMEstimator::calculate_scale_factor) on the device.
//
// Reference: src/optimization/AdaptiveMEstimator.cpp:243-291 (calculate_pko_scale_factor), :294-485 (fit_gmm),
// :710-787 (calculate_js_divergence).  Per GN iteration:
//   1. correspondence count n_c and (iteration 0) the normalisation scale std/6 from the per-block stats
//      that k_correspond wrote (IterativeClosestPointOptimizer.cpp:304-316);
//   2. the GMM sample r_hat[perm[s]], s < min(100, n_c), where perm = std::shuffle(iota(n_c), mt19937(42))
//      is answered from host-built tables (lo_pko_tables.h) and rank -> point via block prefix + ballots;
//   3. k-means (component 0 pinned at 0) + up to 100 EM iterations (fit_gmm);
//   4. JS divergence of the GMM against the normalised Huber kernel for every alpha of the 100-point grid.
//
// Layout on the chip: the EM is a strictly sequential chain of (usually all) 100 iterations, so its latency
// sets the kernel time.  Every workgroup of the launch fits the same GMM redundantly (identical, deterministic
// results, no inter-workgroup traffic).  Inside a workgroup the EM is split by component: wave j evaluates
// only component j's pdf for all samples (ceil(S/64) per lane), the pdfs meet in LDS once per iteration and each
// wave reduces its own component's sums with a permlane/DPP butterfly (gmm_fit_split).  Splitting the SAMPLES
// over waves was measured slower (it adds an LDS exchange without shortening the per-lane exp chains).
// Afterwards workgroup g evaluates the JS divergence for alphas g+1, g+1+G, ... and writes them to global
// memory.  The argmin over the grid (first strict minimum,
// as the reference loop) is taken by the consumers (k_accumulate / k_pko_finish) after the kernel boundary,
// so no in-launch hand-off is needed.
#pragma once
#include "lo_device.h"
#include "lo_math.h"
#include "lo_solve.h"
#include "lo_exact.h"

#include <type_traits>

#include <cfloat>

namespace lo {

__device__ __forceinline__ int pko_sample(const KParams& P, int n, int s) {
    if (n < P.S) return P.small_perm[P.small_off[n] + s];
    const int mode = (n <= 65535) ? ((n & 1) ? 0 : 1) : 2;
    const int lo0 = P.ev_off[mode * (P.S + 1) + s], hi0 = P.ev_off[mode * (P.S + 1) + s + 1];
    int lo = lo0, hi = hi0;                       // last event step <= n - 1
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (P.ev_steps[mid] <= n - 1) lo = mid + 1; else hi = mid;
    }
    return lo == lo0 ? P.base[mode * P.S + s] : P.ev_steps[lo - 1];
}

// gaussian_pdf (AdaptiveMEstimator.cpp:675-685); NaN variances fall through like the reference
__device__ __forceinline__ double gpdf(double x, double mean, double variance) {
    if (variance <= 0.0) return 0.0;
    const double diff = x - mean;
    const double expo = -0.5 * (diff * diff) / variance;
    const double norm = 1.0 / sqrt(2.0 * M_PI * variance);
    return norm * exp(expo);
}

// pko_kernel_weight (AdaptiveMEstimator.cpp:128-156) with tukey_weight / welsch_weight / geman_mcclure_weight /
// pseudo_huber_weight (:99-126), the same operation order; kernel = LO_PKO_* (unknown names map to Cauchy on the host)
__device__ __forceinline__ double pko_kernel_w(double r, double d, int kernel) {
    switch (kernel) {
        case LO_PKO_HUBER: { const double a = fabs(r); return a <= d ? 1.0 : d / a; }
        case LO_PKO_TUKEY: {
            const double a = fabs(r);
            if (a < d) { const double x = a / d, x2 = x * x; return (1 - x2) * (1 - x2); }
            return 0.0;
        }
        case LO_PKO_WELSCH: { const double e2 = r * r, d2 = d * d; return exp(-e2 / d2 / 2.0); }
        case LO_PKO_GEMAN_MCCLURE: { const double e2 = r * r, d2 = d * d; return r * d2 / (d2 + e2) / (d2 + e2); }
        case LO_PKO_PSEUDO_HUBER: { const double e = r, d2 = d * d; return d2 / pow(d2 + e * e, 1.5); }
        default: { const double e2 = r * r, d2 = d * d; return d2 / (d2 + e2); }   // cauchy
    }
}

// Diagnostic build only (-DLO_PKO_STAMPS): workgroup 0 / thread 0 stores s_memtime at phase boundaries
// into DevState::dbg (never read by any other code; the real kernel executes no stamp).
#ifdef LO_PKO_STAMPS
#define LO_STAMP(dbg, i) do { if ((dbg) && threadIdx.x == 0) (dbg)[i] = __builtin_amdgcn_s_memtime(); } while (0)
#define LO_COUNT(dbg, i, v) do { if ((dbg) && threadIdx.x == 0) (dbg)[i] = (v); } while (0)
// a stamp after this wave's outstanding loads have landed
#define LO_STAMP_WAIT(dbg, i, cond)                                                        \
    do {                                                                                   \
        if ((dbg) && (cond)) {                                                             \
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                    \
            (dbg)[i] = __builtin_amdgcn_s_memtime();                                       \
        }                                                                                  \
    } while (0)
#else
#define LO_STAMP(dbg, i) do { } while (0)
#define LO_COUNT(dbg, i, v) do { } while (0)
#define LO_STAMP_WAIT(dbg, i, cond) do { } while (0)
#endif

// exp(y) for y <= 0 or NaN (the E-step exponent -(d^2) * 0.5 / var): Cody-Waite reduction by ln2 and the
// degree-12 Taylor polynomial on |r| <= ln2/2, its tail c3..c12 evaluated by Estrin (r^2, r^4, r^8) and the last
// three steps by Horner, so the dependent chain is 7 FMAs instead of 13 with Horner's accuracy: <= 2 ulp from
// glibc exp over [-745, 0] (checked on 2e7 points; differs from the all-Horner form in 0.08% of them).
// No overflow branch is needed for y <= 0, and the underflow to 0 falls out of v_ldexp_f64.
__device__ __forceinline__ double exp_nonpos(double y) {
    const double n = rint(y * 0x1.71547652b82fep+0);
    double r = fma(-n, 0x1.62e42fefa39efp-1, y);
    r = fma(-n, 0x1.abc9e3b39803fp-56, r);
    const double r2 = r * r, r4 = r2 * r2, r8 = r4 * r4;
    const double q0 = fma(0x1.5555555555555p-5, r, 0x1.5555555555555p-3);     // c3 + c4 r
    const double q1 = fma(0x1.6c16c16c16c17p-10, r, 0x1.1111111111111p-7);    // c5 + c6 r
    const double q2 = fma(0x1.a01a01a01a01ap-16, r, 0x1.a01a01a01a01ap-13);   // c7 + c8 r
    const double q3 = fma(0x1.27e4fb7789f5cp-22, r, 0x1.71de3a556c734p-19);   // c9 + c10 r
    const double q4 = fma(0x1.1eed8eff8d898p-29, r, 0x1.ae64567f544e4p-26);   // c11 + c12 r
    const double s0 = fma(q1, r2, q0), s1 = fma(q3, r2, q2);
    const double tail = fma(q4, r8, fma(s1, r4, s0));
    double p = fma(tail, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    return ldexp(p, static_cast<int>(n));
}

// ---- single-wave reductions ------------------------------------------------------------------------
// Sum of 8 fp64 values over the 64 lanes of a wave without LDS: a butterfly that halves the values per lane
// while halving the lane group (v_permlane32_swap: lanes 32-63 <-> 0-31, v_permlane16_swap: odd <-> even
// 16-lane rows, DPP row_ror:8), after which value q sits in lanes 8q..8q+7; three DPP steps finish each
// 8-lane group and v_readlane broadcasts the totals (wave-uniform results).  ~50 VALU ops, no waits.
__device__ __forceinline__ void pl32_swap(double& a, double& b) {   // a <- [a_lo | b_lo], b <- [a_hi | b_hi]
    const auto lo = __builtin_amdgcn_permlane32_swap(static_cast<unsigned>(__double2loint(a)),
                                                     static_cast<unsigned>(__double2loint(b)), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(static_cast<unsigned>(__double2hiint(a)),
                                                     static_cast<unsigned>(__double2hiint(b)), false, false);
    a = __hiloint2double(static_cast<int>(hi[0]), static_cast<int>(lo[0]));
    b = __hiloint2double(static_cast<int>(hi[1]), static_cast<int>(lo[1]));
}
__device__ __forceinline__ void pl16_swap(double& a, double& b) {   // a <- [a0 b0 a2 b2], b <- [a1 b1 a3 b3] (rows)
    const auto lo = __builtin_amdgcn_permlane16_swap(static_cast<unsigned>(__double2loint(a)),
                                                     static_cast<unsigned>(__double2loint(b)), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(static_cast<unsigned>(__double2hiint(a)),
                                                     static_cast<unsigned>(__double2hiint(b)), false, false);
    a = __hiloint2double(static_cast<int>(hi[0]), static_cast<int>(lo[0]));
    b = __hiloint2double(static_cast<int>(hi[1]), static_cast<int>(lo[1]));
}
__device__ __forceinline__ double readlane64(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}

template <int NV>
__device__ __forceinline__ void wave_totals8(double (&v)[NV]) {
    static_assert(NV >= 1 && NV <= 8, "butterfly handles up to 8 values");
    double u[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) u[q] = q < NV ? v[q] : 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) { pl32_swap(u[q], u[q + 4]); u[q] += u[q + 4]; }   // lo: v_q, hi: v_{q+4}
#pragma unroll
    for (int q = 0; q < 2; ++q) { pl16_swap(u[q], u[q + 2]); u[q] += u[q + 2]; }   // rows: v_q v_{q+2} v_{q+4} v_{q+6}
    const bool up = (threadIdx.x & 8) != 0;
    double t = up ? u[1] : u[0];
    const double o = up ? u[0] : u[1];
    t += dpp64<0x128, 0xf>(o);      // row_ror:8 = lane ^ 8 inside a row -> value q in lanes 8q..8q+7
    t += dpp64<0xB1, 0xf>(t);       // quad_perm [1,0,3,2]
    t += dpp64<0x4E, 0xf>(t);       // quad_perm [2,3,0,1]
    t += dpp64<0x141, 0xf>(t);      // row_half_mirror: 8-lane group total
#pragma unroll
    for (int q = 0; q < NV; ++q) v[q] = readlane64(t, 8 * q);
}

// Up to 4 values with the same pairing tree as wave_totals8 -- lanes (l, l+32), (l, l+16), (l, l+8), then the
// quad and half-row steps -- so each total is bit-identical to wave_totals8's, with half the permlane traffic:
// after the 32- and 16-lane swaps row r holds value r, and one row_ror:8 replaces the half-row selects.
template <int NV>
__device__ __forceinline__ void wave_totals4(double (&v)[NV]) {
    static_assert(NV >= 1 && NV <= 4, "butterfly handles up to 4 values");
    double u[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) u[q] = q < NV ? v[q] : 0.0;
#pragma unroll
    for (int q = 0; q < 2; ++q) { pl32_swap(u[q], u[q + 2]); u[q] += u[q + 2]; }   // lo: v_q, hi: v_{q+2}
    pl16_swap(u[0], u[1]);
    double t = u[0] + u[1];         // row r: value r
    t += dpp64<0x128, 0xf>(t);      // row_ror:8
    t += dpp64<0xB1, 0xf>(t);       // quad_perm [1,0,3,2]
    t += dpp64<0x4E, 0xf>(t);       // quad_perm [2,3,0,1]
    t += dpp64<0x141, 0xf>(t);      // row_half_mirror: 8-lane group total
#pragma unroll
    for (int q = 0; q < NV; ++q) v[q] = readlane64(t, 16 * q);
}

// fit_gmm (AdaptiveMEstimator.cpp:294-485) with the EM split over the workgroup's waves: wave j < K owns
// component j (every lane computes ONE pdf per sample instead of K), the per-sample pdfs meet in LDS (s_p) and
// the summed |d mean| of components >= 1 in s_dm, one barrier per iteration.  Per-lane sample mapping (sample s*64 + lane), the order of the
// per-sample sum (((0 + p_0) + p_1) + p_2), the per-lane accumulation order and the butterfly tree do not
// depend on the split (the fitted GMM is bit-identical to a single wave doing all components), with a third of
// the VALU issue on the critical path.  k-means and the initial variance run redundantly in every wave (identical inputs and code,
// so identical results, no exchange).  All NW waves execute the loop (waves >= K only join the barriers), and
// the convergence test reads the same LDS values everywhere, so every wave leaves at the same iteration.
// emst (nullable, one workgroup): s_memtime cycles of the EM loop, its iterations and one fit are added there.
template <int K, int SPL>
__device__ __forceinline__ void gmm_fit_split(const double* s_sd, int S, const int32_t* draws, double* gmm,
                                              double* s_p, double* s_dm, unsigned long long* dbg,
                                              unsigned long long* emst) {
    static_assert(3 * K - 1 <= 8, "partials");
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int j = wid < K ? wid : -1;                      // this wave's component (-1: barriers only)
    if (j < 0) {
        // a wave without a component only follows the barriers and the change test (no VALU work that would compete
        // for issue with a component wave on the same SIMD in workgroups of more than 4 waves)
        __syncthreads();
        int buf = 0;
#if defined(LO_XC_EXP) && LO_XC_EXP == 3
        for (int em = 0; em < 1; ++em) {
#else
        for (int em = 0; em < 100; ++em) {
#endif
            __syncthreads();
            double change = 0.0;
#pragma unroll
            for (int q = 1; q < K; ++q) change += s_dm[buf * kMaxK + q];
            if (change < 1e-6) break;
            buf ^= 1;
        }
        return;
    }
    double x[SPL];
    bool have[SPL];
#pragma unroll
    for (int s = 0; s < SPL; ++s) {
        have[s] = lane + 64 * s < S;
        x[s] = have[s] ? s_sd[lane + 64 * s] : 0.0;
    }
    double mu[K], cnt[K];
    mu[0] = 0.0;
#pragma unroll
    for (int q = 1; q < K; ++q) mu[q] = s_sd[draws[q - 1]];
#pragma unroll
    for (int q = 0; q < K; ++q) cnt[q] = 0.0;
    // ---- k-means until the means repeat exactly (:351-389) ----
    // Component 0's mean is pinned, so only its count is needed, and counts are small integers (exact in fp64):
    // it is S minus the others' counts, and the 2(K - 1) remaining totals fit the 4-value butterfly (each total
    // bit-identical to wave_totals8's, so the fit still equals gmm_fit_1w's).
    for (int guard = 0; guard < 100000; ++guard) {
        double v[2 * K - 1];
#pragma unroll
        for (int q = 0; q < 2 * K - 1; ++q) v[q] = 0.0;
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
            double md = DBL_MAX;
            int ci = 0;
#pragma unroll
            for (int q = 0; q < K; ++q) { const double d = fabs(x[s] - mu[q]); if (d < md) { md = d; ci = q; } }
#pragma unroll
            for (int q = 1; q < K; ++q) {
                const bool mine = have[s] && ci == q;
                v[q] += mine ? 1.0 : 0.0;
                v[K + q - 1] += mine ? x[s] : 0.0;
            }
        }
        if constexpr (K > 1) {
            double u[2 * K - 2];
#pragma unroll
            for (int q = 0; q < 2 * K - 2; ++q) u[q] = v[q + 1];
            wave_totals4<2 * K - 2>(u);
#pragma unroll
            for (int q = 0; q < 2 * K - 2; ++q) v[q + 1] = u[q];
        }
        v[0] = static_cast<double>(S);
#pragma unroll
        for (int q = 1; q < K; ++q) v[0] -= v[q];
        bool eq = true;
        double nm[K];
#pragma unroll
        for (int q = 0; q < K; ++q) {
            nm[q] = (q == 0) ? 0.0 : (v[q] > 0.0 ? v[K + q - 1] / v[q] : 0.0);
            eq = eq && (nm[q] == mu[q]);
            cnt[q] = v[q];
        }
        LO_COUNT(dbg, 9, guard + 1);
        if (eq) break;
#pragma unroll
        for (int q = 0; q < K; ++q) mu[q] = nm[q];
    }
    LO_STAMP(dbg, 3);
    double m1 = 0.0;
#pragma unroll
    for (int s = 0; s < SPL; ++s) m1 += have[s] ? x[s] : 0.0;
    const double mean = wave_total(m1) / S;
    double m2 = 0.0;
#pragma unroll
    for (int s = 0; s < SPL; ++s) m2 += have[s] ? (x[s] - mean) * (x[s] - mean) : 0.0;
    const double iv = wave_total(m2) / S;
    const double invS = 1.0 / static_cast<double>(S);
    constexpr double kInvSqrt2Pi = 0.3989422804014327;
    // this wave's component state
    const int jj = j < 0 ? 0 : j;
    double muj = mu[0], cntj = cnt[0];
#pragma unroll
    for (int q = 1; q < K; ++q) if (jj == q) { muj = mu[q]; cntj = cnt[q]; }
    double wj = cntj / static_cast<double>(S), varj = iv;
    const double rs0 = rsq64(iv);
    double ca = (iv <= 0.0) ? 0.0 : wj * (rs0 * kInvSqrt2Pi);
    double cb = (iv <= 0.0) ? 0.0 : 0.5 * (rs0 * rs0);
    LO_STAMP(dbg, 4);
    const unsigned long long em_t0 = emst ? __builtin_amdgcn_s_memtime() : 0ull;

    // One barrier per iteration: after its M-step each wave evaluates the NEXT iteration's pdfs with the updated
    // parameters (speculatively) into the other half of the double-buffered s_p / s_dm, then the barrier; if
    // the change test then ends the EM, the speculative pdfs are simply dropped (the parameters are those of
    // the converged M-step, as the reference's loop leaves them).
    constexpr int kStride = 64 * SPL;                      // s_p[buffer][component][sample]
    constexpr int kBuf = K * kStride;
    double p[SPL], d[SPL];
#pragma unroll
    for (int s = 0; s < SPL; ++s) {
        d[s] = x[s] - muj;
        p[s] = ca * exp_nonpos(-((d[s] * d[s]) * cb));
        if (j >= 0) s_p[j * kStride + 64 * s + lane] = p[s];
    }
    __syncthreads();
    // every component's pdfs of the current iteration, read right after the barrier TOGETHER with the change test's
    // s_dm values (one LDS round trip per iteration instead of two: the compare no longer gates these reads)
    double pv[K][SPL];
#pragma unroll
    for (int q = 0; q < K; ++q)
#pragma unroll
        for (int s = 0; s < SPL; ++s) pv[q][s] = s_p[q * kStride + 64 * s + lane];
    int n_em = 100;
#if defined(LO_XC_EXP) && LO_XC_EXP == 3
    constexpr int kEmMax = 1;                              // diagnostic: one EM iteration (the launch without its EM)
#else
    constexpr int kEmMax = 100;
#endif
    // One EM iteration with the double buffer's half as a compile-time constant (the loop below runs them in pairs):
    // the next pdfs' LDS reads then sit at immediate offsets from one lane base (ds_read2st64_b64 pairs) instead of
    // per-read address arithmetic on a runtime buffer index -- that arithmetic, and the split reads it brought, were
    // the EM's 1092 -> 1152-cycle drift between rounds 3 and 5 (scripts/pko_em_isa.py, same source, different
    // codegen).  Returns true when the change test ends the EM.
    auto em_step = [&](auto bc, int em) -> bool {
        constexpr int buf = decltype(bc)::value;
        double v[3] = {0.0, 0.0, 0.0};                     // N_j | sum r x | sum r d^2
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
            double sr = pv[0][s];                          // pdfs are >= +0 (or NaN): 0 + p_0 == p_0
#pragma unroll
            for (int q = 1; q < K; ++q) sr += pv[q][s];
            const double isr = have[s] ? rcp64_1n(sr) : 0.0;
            const double r = p[s] * isr;
            // the first sample's terms start the sums (no "0 + t": r >= +0, so only the sign of an all-zero
            // total could differ, and no value downstream depends on it)
            v[0] = s == 0 ? r : v[0] + r;
            v[1] = s == 0 ? r * x[s] : v[1] + r * x[s];
            v[2] = s == 0 ? (r * d[s]) * d[s] : v[2] + (r * d[s]) * d[s];
        }
        wave_totals4<3>(v);
        const double Nk = v[0];
        const double iN = rcp64_1n(Nk);
        const double nmu = (jj == 0) ? 0.0 : v[1] * iN;
        const double dm = nmu - muj;
        double nv = v[2] * iN - dm * dm;
        nv = (nv < 1e-6) ? 1e-6 : nv;                      // std::max(nv, 1e-6), NaN preserved
        wj = Nk * invS;
        muj = nmu;
        varj = nv;
        const double rs = rsq64_1n(nv);
        ca = wj * (rs * kInvSqrt2Pi);
        cb = 0.5 * (rs * rs);
        if (j >= 1 && lane == 0) s_dm[buf * kMaxK + j] = fabs(dm);
        double* spn = s_p + (buf ^ 1) * kBuf;              // speculative E-step of iteration em + 1
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
            d[s] = x[s] - muj;
            p[s] = ca * exp_nonpos(-((d[s] * d[s]) * cb));
            if (j >= 0) spn[j * kStride + 64 * s + lane] = p[s];
        }
        __syncthreads();
        double dmv[kMaxK];
#pragma unroll
        for (int q = 1; q < K; ++q) dmv[q] = s_dm[buf * kMaxK + q];
#pragma unroll
        for (int q = 0; q < K; ++q)
#pragma unroll
            for (int s = 0; s < SPL; ++s) pv[q][s] = spn[q * kStride + 64 * s + lane];
        // pin the pdf reads above the exit branch (the compiler would otherwise sink them below it, behind the
        // s_dm round trip)
#pragma unroll
        for (int q = 0; q < K; ++q)
#pragma unroll
            for (int s = 0; s < SPL; ++s) asm volatile("" : "+v"(pv[q][s]));
        double change = 0.0;
#pragma unroll
        for (int q = 1; q < K; ++q) change += dmv[q];
        LO_COUNT(dbg, 8, em + 1);
        if (change < 1e-6) { n_em = em + 1; return true; }
        return false;
    };
    for (int em = 0; em < kEmMax; em += 2) {
        if (em_step(std::integral_constant<int, 0>{}, em)) break;
        if (em + 1 >= kEmMax || em_step(std::integral_constant<int, 1>{}, em + 1)) break;
    }
    LO_STAMP(dbg, 5);
    if (emst && threadIdx.x == 0) {                        // wave 0 (component 0): the loop's own clock
        atomicAdd(emst, __builtin_amdgcn_s_memtime() - em_t0);
        atomicAdd(emst + 1, static_cast<unsigned long long>(n_em));
        atomicAdd(emst + 2, 1ull);
    }
    if (j >= 0 && lane == 0) { gmm[j] = wj; gmm[K + j] = muj; gmm[2 * K + j] = varj; }
}

// Batched launches: the whole fit on ONE wave (all K components), bit-identical to gmm_fit_split -- the same
// per-sample sum (((0 + p_0) + p_1) + p_2), per-lane accumulation order and butterfly tree per value (the tree a
// value goes through in wave_totals8 does not depend on its slot).  A batch is bound by fp64 issue, not by the
// EM's latency: one wave drops the two extra butterflies, reciprocals and pdf exchanges the split pays per
// iteration, and no other wave replicates k-means.
template <int K, int SPL>
__device__ __forceinline__ void gmm_fit_1w(const double* s_sd, int S, const int32_t* draws, double* gmm) {
    static_assert(3 * K - 1 <= 8, "partials");
    const int lane = threadIdx.x & 63;
    double x[SPL];
    bool have[SPL];
#pragma unroll
    for (int s = 0; s < SPL; ++s) {
        have[s] = lane + 64 * s < S;
        x[s] = have[s] ? s_sd[lane + 64 * s] : 0.0;
    }
    double mu[K], cnt[K];
    mu[0] = 0.0;
#pragma unroll
    for (int q = 1; q < K; ++q) mu[q] = s_sd[draws[q - 1]];
#pragma unroll
    for (int q = 0; q < K; ++q) cnt[q] = 0.0;
    for (int guard = 0; guard < 100000; ++guard) {            // k-means as gmm_fit_split
        double v[2 * K - 1];
#pragma unroll
        for (int q = 0; q < 2 * K - 1; ++q) v[q] = 0.0;
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
            double md = DBL_MAX;
            int ci = 0;
#pragma unroll
            for (int q = 0; q < K; ++q) { const double d = fabs(x[s] - mu[q]); if (d < md) { md = d; ci = q; } }
#pragma unroll
            for (int q = 0; q < K; ++q) {
                const bool mine = have[s] && ci == q;
                v[q] += mine ? 1.0 : 0.0;
                if (q > 0) v[K + q - 1] += mine ? x[s] : 0.0;
            }
        }
        wave_totals8<2 * K - 1>(v);
        bool eq = true;
        double nm[K];
#pragma unroll
        for (int q = 0; q < K; ++q) {
            nm[q] = (q == 0) ? 0.0 : (v[q] > 0.0 ? v[K + q - 1] / v[q] : 0.0);
            eq = eq && (nm[q] == mu[q]);
            cnt[q] = v[q];
        }
        if (eq) break;
#pragma unroll
        for (int q = 0; q < K; ++q) mu[q] = nm[q];
    }
    double m1 = 0.0;
#pragma unroll
    for (int s = 0; s < SPL; ++s) m1 += have[s] ? x[s] : 0.0;
    const double mean = wave_total(m1) / S;
    double m2 = 0.0;
#pragma unroll
    for (int s = 0; s < SPL; ++s) m2 += have[s] ? (x[s] - mean) * (x[s] - mean) : 0.0;
    const double iv = wave_total(m2) / S;
    const double invS = 1.0 / static_cast<double>(S);
    constexpr double kInvSqrt2Pi = 0.3989422804014327;
    double w[K], var[K], ca[K], cb[K];
    const double rs0 = rsq64(iv);
#pragma unroll
    for (int q = 0; q < K; ++q) {
        w[q] = cnt[q] / static_cast<double>(S);
        var[q] = iv;
        ca[q] = (iv <= 0.0) ? 0.0 : w[q] * (rs0 * kInvSqrt2Pi);
        cb[q] = (iv <= 0.0) ? 0.0 : 0.5 * (rs0 * rs0);
    }
    double p[K][SPL], d[K][SPL];
#pragma unroll
    for (int q = 0; q < K; ++q)
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
            d[q][s] = x[s] - mu[q];
            p[q][s] = ca[q] * exp_nonpos(-((d[q][s] * d[q][s]) * cb[q]));
        }
    for (int em = 0; em < 100; ++em) {
        double v[3 * K - 1];                                  // N_q | sum r x (q >= 1) | sum r d^2
#pragma unroll
        for (int q = 0; q < 3 * K - 1; ++q) v[q] = 0.0;
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
            double sr = p[0][s];                           // as gmm_fit_split: 0 + p_0 == p_0
#pragma unroll
            for (int q = 1; q < K; ++q) sr += p[q][s];
            const double isr = have[s] ? rcp64_1n(sr) : 0.0;
#pragma unroll
            for (int q = 0; q < K; ++q) {
                const double r = p[q][s] * isr;       // first sample starts the sums, as gmm_fit_split
                v[q] = s == 0 ? r : v[q] + r;
                if (q > 0) v[K + q - 1] = s == 0 ? r * x[s] : v[K + q - 1] + r * x[s];
                v[2 * K - 1 + q] = s == 0 ? (r * d[q][s]) * d[q][s] : v[2 * K - 1 + q] + (r * d[q][s]) * d[q][s];
            }
        }
        wave_totals8<3 * K - 1>(v);
        double change = 0.0;
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const double Nk = v[q];
            const double iN = rcp64_1n(Nk);
            const double nmu = (q == 0) ? 0.0 : v[K + q - 1] * iN;
            const double dm = nmu - mu[q];
            double nv = v[2 * K - 1 + q] * iN - dm * dm;
            nv = (nv < 1e-6) ? 1e-6 : nv;
            w[q] = Nk * invS;
            mu[q] = nmu;
            var[q] = nv;
            const double rs = rsq64_1n(nv);
            ca[q] = w[q] * (rs * kInvSqrt2Pi);
            cb[q] = 0.5 * (rs * rs);
            if (q >= 1) change += fabs(dm);
        }
        if (change < 1e-6) break;
#pragma unroll
        for (int q = 0; q < K; ++q)
#pragma unroll
            for (int s = 0; s < SPL; ++s) {
                d[q][s] = x[s] - mu[q];
                p[q][s] = ca[q] * exp_nonpos(-((d[q][s] * d[q][s]) * cb[q]));
            }
    }
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < K; ++q) { gmm[q] = w[q]; gmm[K + q] = mu[q]; gmm[2 * K + q] = var[q]; }
    }
}

template <int K>
__device__ __forceinline__ void gmm_fit_dispatch(const double* s_sd, int S, const int32_t* draws, double* gmm,
                                                 double* s_p, double* s_dm, unsigned long long* dbg,
                                                 unsigned long long* emst) {
    if (S <= 64) gmm_fit_split<K, 1>(s_sd, S, draws, gmm, s_p, s_dm, dbg, emst);
    else if (S <= 128) gmm_fit_split<K, 2>(s_sd, S, draws, gmm, s_p, s_dm, dbg, emst);
    else gmm_fit_split<K, 4>(s_sd, S, draws, gmm, s_p, s_dm, dbg, emst);
}

template <int K>
__device__ __forceinline__ void gmm_fit_1w_dispatch(const double* s_sd, int S, const int32_t* draws, double* gmm) {
    if ((threadIdx.x >> 6) != 0) return;                  // wave 0 fits; any other wave goes on to the barrier
    if (S <= 64) gmm_fit_1w<K, 1>(s_sd, S, draws, gmm);
    else if (S <= 128) gmm_fit_1w<K, 2>(s_sd, S, draws, gmm);
    else gmm_fit_1w<K, 4>(s_sd, S, draws, gmm);
}

// Speculative normal equations (single-scan launches of small scans, nb_acc <= kFuseMaxBlocks).  The accumulate
// pass depends on the PKO only through the Huber delta, one of NA + 1 values (alphas[1..NA], or min_scale when no
// JS cost is finite).  Workgroups G, G+1, ... of the PKO launch evaluate every candidate while the GMM fit runs,
// and k_solve_pick reduces the selected one: the accumulate leaves the iteration's critical path.  Workgroup wgi
// takes candidate wgi / W (W = ceil(nb_acc / kSpecBlocksPerWG)) and its kSpecBlocksPerWG 256-point blocks
// starting at kSpecBlocksPerWG * (wgi % W); each block's partial is formed exactly as accumulate_body forms it
// (one point per thread, fp32 wave_total, fp64 sum over the 4 waves), so the solve is bit-identical.
// The normal-equation partials of blocks [vb0, vb1) with Huber delta dl into dst[vb][kNE], each block's partial formed
// exactly as accumulate_body forms it (one point per thread, fp32 wave_total, fp64 sum over the 4 waves).  SC1: the
// partials are stored through Mem<true>, for a reader in another workgroup of the same launch.
template <bool SC1>
__device__ void acc_blocks(const KParams& P, const int32_t* slot, const float (&T)[12], double scale, float dl, int vb0,
                           int vb1, double* dst) {
    __shared__ float s_acc[kWavesPerBlock][kNE];
    const int tid = threadIdx.x, wid = tid >> 6;
    const int n = scan_n(P);
    if (!P.kd_res) {
        // surfel path, software-pipelined: block vb + 2's slot index and block vb + 1's point and surfel are loaded
        // while block vb is accumulated (the slot -> surfel chain otherwise costs two round trips per block); the
        // terms (acc_terms) and the reductions are exactly the per-block ones below, so the partials are the same bits
        auto slot_of = [&](int vb) { const int i = vb * kBlock + tid; return (vb < vb1 && i < n) ? slot[i] : -1; };
        int s1 = slot_of(vb0), s2 = slot_of(vb0 + 1);
        float px = 0.0f, py = 0.0f, pz = 0.0f;
        Slot sl{};
        if (s1 >= 0) {
            const int i = vb0 * kBlock + tid;
            px = P.pts[3 * i]; py = P.pts[3 * i + 1]; pz = P.pts[3 * i + 2];
            sl = P.tab[s1];
        }
        for (int vb = vb0; vb < vb1; ++vb) {
            const int s0 = s1;
            const float cx = px, cy = py, cz = pz;
            const Slot cs = sl;
            s1 = s2;
            s2 = slot_of(vb + 2);
            if (s1 >= 0) {
                const int i = (vb + 1) * kBlock + tid;
                px = P.pts[3 * i]; py = P.pts[3 * i + 1]; pz = P.pts[3 * i + 2];
                sl = P.tab[s1];
            }
            float acc[kNE];
#pragma unroll
            for (int k = 0; k < kNE; ++k) acc[k] = 0.0f;
            if (s0 >= 0) {
                float wx, wy, wz;
                transform_pt(T, cx, cy, cz, wx, wy, wz);
                acc_terms(P, T, scale, dl, residual_f64(cs, wx, wy, wz), cx, cy, cz, cs, acc);
            }
            wave_totals_f32<kNE>(acc, s_acc[wid]);
            __syncthreads();
            if (tid < kNE) {
                double v = 0.0;
#pragma unroll
                for (int w = 0; w < kWavesPerBlock; ++w) v += static_cast<double>(s_acc[w][tid]);
                Mem<SC1>::st(dst + static_cast<size_t>(vb) * kNE + tid, v);
            }
            __syncthreads();
        }
        return;
    }
    for (int vb = vb0; vb < vb1; ++vb) {
        float acc[kNE];
#pragma unroll
        for (int k = 0; k < kNE; ++k) acc[k] = 0.0f;
        const int i = vb * kBlock + tid;
        if (i < n) acc_point(P, slot, T, scale, dl, i, acc);
        wave_totals_f32<kNE>(acc, s_acc[wid]);
        __syncthreads();
        if (tid < kNE) {
            double v = 0.0;
#pragma unroll
            for (int w = 0; w < kWavesPerBlock; ++w) v += static_cast<double>(s_acc[w][tid]);
            Mem<SC1>::st(dst + static_cast<size_t>(vb) * kNE + tid, v);
        }
        __syncthreads();
    }
}
__device__ __forceinline__ float cand_delta(const KParams& P, int c) {
    return static_cast<float>(c < P.NA ? P.alphas[c + 1] : P.min_scale);
}
// Candidate workgroup wgi: part (wgi % W) of candidate c = wgi / W's partials.  With P.cand_rec the candidate's GN step
// is also solved here, while the EM still runs (:417-448: solve_sums + solve_step over the same partials the fused
// k_accumulate / k_solve_pick would reduce, so the same bits): W = 1 in this workgroup; W > 1 by the candidate's last
// workgroup to arrive -- the parts' partials are stored write-through and drained before an agent-scope add on the
// candidate's counter (MI355X_MICROARCH.md "inter-workgroup visibility", the one-lane-signals row), and the last
// arrival reads them past L1 and re-zeroes the counter for the next launch.  The record [kCandWords] is read by
// k_pick_correspond / k_pick after the launch, so the selected solve leaves the iteration's critical path.
__device__ void acc_candidate(const KParams& P, double scale, int wgi) {
#ifdef LO_PKO_STAMPS
    const unsigned long long c_t0 = __builtin_amdgcn_s_memtime();
#endif
    const int nb = P.nb_acc;
    const int W = (nb + kSpecBlocksPerWG - 1) / kSpecBlocksPerWG;
    const int c = wgi / W, part = wgi - c * W;
    if (c > P.NA) return;
    const int tid = threadIdx.x;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = P.st->pose[k];
    double* part_c = P.acc_part + static_cast<size_t>(c) * kFuseMaxBlocks * kNE;
    const int vb0 = part * kSpecBlocksPerWG, vb1 = min(nb, (part + 1) * kSpecBlocksPerWG);
    const bool handoff = P.cand_rec && W > 1;
    if (handoff) acc_blocks<true>(P, P.slot, T, scale, cand_delta(P, c), vb0, vb1, part_c);
    else acc_blocks<false>(P, P.slot, T, scale, cand_delta(P, c), vb0, vb1, part_c);
    if (!P.cand_rec) return;
    __shared__ int s_last;
    __shared__ double s_tot[kNE];
    __shared__ float s_rec[kCandWords];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // every storing wave: its partials have left
    __syncthreads();
    if (handoff) {
        if (tid == 0) {
            unsigned* cnt = P.cand_cnt + c;
            const unsigned old = __hip_atomic_fetch_add((g_u32*)(cnt), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = old + 1u == static_cast<unsigned>(W) ? 1 : 0;
            if (s_last) Mem<true>::st(cnt, 0u);               // every part has arrived: ready for the next launch
        }
        __syncthreads();
        if (!s_last) return;
        solve_sums<kBlock, true>(part_c, nb, s_tot);
    } else {
        solve_sums<kBlock, false>(part_c, nb, s_tot);
    }
    if (tid == 0) {
        float Tn[12];
        lo_iter_log lg;
        const bool conv = solve_step(P, s_tot, T, Tn, &lg);
#pragma unroll
        for (int q = 0; q < 12; ++q) s_rec[q] = Tn[q];
        s_rec[kCandCost] = lg.cost;
#pragma unroll
        for (int q = 0; q < 21; ++q) s_rec[kCandH + q] = lg.H[q];
#pragma unroll
        for (int q = 0; q < 6; ++q) { s_rec[kCandG + q] = lg.g[q]; s_rec[kCandD + q] = lg.delta[q]; }
        s_rec[kCandConv] = conv ? 1.0f : 0.0f;
        s_rec[kCandConv + 1] = 0.0f;
    }
    __syncthreads();
    if (tid < kCandWords) P.cand_rec[static_cast<size_t>(c) * kCandWords + tid] = s_rec[tid];
#ifdef LO_PKO_STAMPS
    if (tid == 0) {                          // diagnostic: the slowest candidate workgroup's cycles (dbg[15])
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        atomicMax(&P.st->dbg[15], __builtin_amdgcn_s_memtime() - c_t0);
        if (c == 0) P.st->dbg[7] = __builtin_amdgcn_s_memtime() - c_t0;
    }
#endif
}

// Reference-exact candidates (lo_set_exact, scans with nb_acc <= kFuseMaxBlocks): candidate c's GN step exactly as the
// reference forms it -- the 43 running fp32 sums of build_ne in correspondence (scan) order (:345-410), Eigen's fp32
// LDLT and the re-projected update (:417-448; lo_exact.h) -- in ONE workgroup while the EM runs, written as the same
// 48-word record acc_candidate writes, so k_pick_correspond / k_pick take it unchanged.
// exact_sums_wg: the 43 sequential sums of build_ne with Huber delta dl at pose T into s_tot (LDS), by one 256-thread
// workgroup; dyn: kXcLdsBytes of LDS; every thread calls it.  Per chunk of 192 points, waves 1-3 form each accepted
// point's 14 factors (exact_point_factors: J, wJ, wr, r) and stage them factor-major in LDS, compacted over the whole
// chunk in point order (each region's valid count is published one chunk ahead, from the slot indices the producers
// hold two chunks ahead) and padded with zero factors to a multiple of 16 rows; wave 0's lane k forms term k of every
// staged row as fa * fb (the same fp32 product build_ne forms) and adds it to its running sum, one rounding per
// addition, a chunk behind the producers (double-buffered, one barrier per chunk).  A zero pad row adds +0, which
// leaves a running sum unchanged: the sums start at +0 and never become -0 (x + -x rounds to +0).  The consumer's loop
// is uniform (no per-row test), three groups of 16 rows in flight (xc_add_mul).
// The consumer's stages: XcRows = 16 staged rows of a lane's two factors, XcProd = their 16 fp32 products (each the
// same separately rounded a * b; v_pk_mul_f32 rounds each half on its own).  xc_add_mul adds a group's products in row
// order and places one packed product of the next group between every two adds (sched_barrier): the in-order wave
// issues it in the dependent add's latency.  scripts/consumer_microbench.hip V5: 167 cycles per 16 rows against 199
// for the read-ahead loop this replaces (floor 16 x 8.6 = 138, profiles/r06_consumer_microbench_v5.txt).
typedef float xc_f2 __attribute__((ext_vector_type(2)));
struct XcRows { float4 a[4], b[4]; };
struct XcProd { xc_f2 v[8]; };
__device__ __forceinline__ void xc_read(XcRows& r, const float4* A, const float4* B, int g) {
#pragma unroll
    for (int q = 0; q < 4; ++q) { r.a[q] = A[4 * g + q]; r.b[q] = B[4 * g + q]; }
}
__device__ __forceinline__ xc_f2 xc_mul(const XcRows& c, int i) {   // products 2i, 2i + 1 of the group
    const float4 a = c.a[i >> 1], b = c.b[i >> 1];
    return (i & 1) ? xc_f2{a.z, a.w} * xc_f2{b.z, b.w} : xc_f2{a.x, a.y} * xc_f2{b.x, b.y};
}
__device__ __forceinline__ void xc_add_mul(float& sum, const XcProd& p, XcProd& pn, const XcRows& c) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        sum += p.v[i].x;
        __builtin_amdgcn_sched_barrier(0);
        pn.v[i] = xc_mul(c, i);
        __builtin_amdgcn_sched_barrier(0);
        sum += p.v[i].y;
        __builtin_amdgcn_sched_barrier(0);
    }
}

__device__ void exact_sums_wg(const KParams& P, const float (&T)[12], double scale, float dl, float* dyn, float* s_tot) {
    float* s_f = dyn;                                      // [2][kXcFactors][kXcStride]
    int* s_cnt = reinterpret_cast<int*>(dyn + kXcCntOff);  // [4][kXcRegions]
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, r = wid - 1;
    const int n = scan_n(P);
    const int nch = (n + kXcChunk - 1) / kXcChunk;
    __syncthreads();                                       // earlier uses of the dynamic buffer are over
    // producer state: this lane's point of the current chunk (loaded) and the slot of the next
    int sl_cur = -1, sl_nxt = -1;
    float px = 0.0f, py = 0.0f, pz = 0.0f;
    Slot sv{};
    double rv = 0.0;
    auto pidx = [&](int ch) { return ch * kXcChunk + r * kWave + lane; };
    // global (not flat) loads: a flat load in flight would hold up every LDS wait of the chunk (gld)
    const double* res = P.kd_res ? P.kd_res : P.res_out;   // the stored fp64 residual (same bits as recomputing)
    auto slot_at = [&](int ch) { const int i = pidx(ch); return (ch < nch && i < n) ? gld(P.slot + i) : -1; };
    auto load_pt = [&](int ch, int s) {
        if (s >= 0) {
            const int i = pidx(ch);
            px = gld(P.pts + 3 * i); py = gld(P.pts + 3 * i + 1); pz = gld(P.pts + 3 * i + 2);
            sv = gld_slot(P.tab + s);
            rv = gld(res + i);
        }
    };
    if (wid > 0) {
        sl_cur = slot_at(0);
        sl_nxt = slot_at(1);
        load_pt(0, sl_cur);
        const int c0 = __popcll(__ballot(sl_cur >= 0));
        if (lane == 0) s_cnt[r] = c0;                      // chunk 0's region counts (buffer 0)
    }
    // consumer: lane k's factor rows (lanes >= 43 are masked off in the add loop)
    int fa, fb;
    exact_term_factors(lane < kExactTerms ? lane : 0, fa, fb);
    __syncthreads();
    float sum = 0.0f;                                      // consumer: lane k's running sum of term k
#ifdef LO_PKO_STAMPS
    unsigned long long t_work = 0, t_wait = 0;             // diagnostic: this wave's cycles in its part / at the barrier
#endif
    for (int ch = 0; ch <= nch; ++ch) {
#ifdef LO_PKO_STAMPS
        const unsigned long long t_c0 = __builtin_amdgcn_s_memtime();
#endif
        if (wid > 0 && ch < nch) {
            float* buf = s_f + (ch & 1) * kXcBuf;
            const int* cn = s_cnt + (ch & 3) * kXcRegions;
            const int c0 = cn[0], c1 = cn[1], tot = c0 + c1 + cn[2];
            const int off = r == 0 ? 0 : (r == 1 ? c0 : c0 + c1);
            const bool valid = sl_cur >= 0;
            const uint64_t m = __ballot(valid);
#if defined(LO_XC_EXP) && LO_XC_EXP == 1
            if (false) {                                   // diagnostic: producers skip the factors (consumer alone)
#else
            if (valid) {
#endif
                float f[kXcFactors];
                exact_point_factors(P, T, scale, dl, rv, px, py, pz, sv, f);
                const int row = off + __popcll(m & ((1ull << lane) - 1ull));
#pragma unroll
                for (int j = 0; j < kXcFactors; ++j) buf[j * kXcStride + row] = f[j];
            }
            const int pad = ((tot + kXcPad - 1) & ~(kXcPad - 1)) - tot;
            if (r == kXcRegions - 1 && lane < pad) {       // zero factor rows up to the next multiple of 16
#pragma unroll
                for (int j = 0; j < kXcFactors; ++j) buf[j * kXcStride + tot + lane] = 0.0f;
            }
            // the next chunk's point / surfel / residual, the slot of the one after, and the next chunk's count
            sl_cur = sl_nxt;
            sl_nxt = slot_at(ch + 2);
            load_pt(ch + 1, sl_cur);
            const int cn1 = __popcll(__ballot(sl_cur >= 0));
            if (lane == 0) s_cnt[((ch + 1) & 3) * kXcRegions + r] = cn1;
#if defined(LO_XC_EXP) && LO_XC_EXP == 2
        } else if (false) {                                // diagnostic: no adds (producers alone)
#else
        } else if (wid == 0 && ch > 0 && lane < kExactTerms) {   // lanes 43-63 stay masked off: a third less LDS traffic
#endif
            const float* base = s_f + ((ch - 1) & 1) * kXcBuf;
            const float4* A = reinterpret_cast<const float4*>(base + fa * kXcStride);
            const float4* B = reinterpret_cast<const float4*>(base + fb * kXcStride);
            const int* cn = s_cnt + ((ch - 1) & 3) * kXcRegions;
            const int ng = (cn[0] + cn[1] + cn[2] + kXcPad - 1) / kXcPad;   // groups of 16 rows (uniform)
            if (ng > 0) {
                // three stages: the products of group g (p), the rows of group g + 1 (c), the reads of group g + 2;
                // the products of g + 1 are formed one v_pk_mul_f32 between every two adds of g, in the adds' latency
                // (two steps per trip with the register sets swapped, so no stage is copied and no read is waited
                // for before its use; reads stay within the staged groups)
                XcRows c0, c1;
                XcProd p0, p1;
                xc_read(c0, A, B, 0);
#pragma unroll
                for (int i = 0; i < 8; ++i) p0.v[i] = xc_mul(c0, i);
                xc_read(c0, A, B, ng > 1 ? 1 : 0);
                // (whole trips only: products a break would leave unused get sunk past the break by the compiler,
                // out of the adds' latency; an odd last group is added after the loop)
                int g = 0;
                for (; g + 2 <= ng; g += 2) {
                    xc_read(c1, A, B, g + 2 < ng ? g + 2 : ng - 1);
                    xc_add_mul(sum, p0, p1, c0);               // group g's adds, group g + 1's products
                    xc_read(c0, A, B, g + 3 < ng ? g + 3 : ng - 1);
                    xc_add_mul(sum, p1, p0, c1);               // group g + 1's adds, group g + 2's products
                }
                if (g < ng) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) { sum += p0.v[i].x; sum += p0.v[i].y; }
                }
            }
        }
#ifdef LO_PKO_STAMPS
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const unsigned long long t_c1 = __builtin_amdgcn_s_memtime();
        __syncthreads();
        const unsigned long long t_c2 = __builtin_amdgcn_s_memtime();
        t_work += t_c1 - t_c0;
        t_wait += t_c2 - t_c1;
#else
        __syncthreads();
#endif
    }
#ifdef LO_PKO_STAMPS
    // diagnostic sums over every exact candidate of the launch: dbg[16] calls, dbg[17] / [18] the consumer wave's add /
    // barrier cycles, dbg[19] / [20] producer wave 1's term / barrier cycles (lo_debug_counters_ex)
#ifdef LO_PKO_SUMS_COUNTERS                  // (r05's per-call counters; dbg[16..18] hold the r06 timeline stamps)
    if (lane == 0 && wid == 0) {
        atomicAdd(&P.st->dbg[16], 1ull);
        atomicAdd(&P.st->dbg[17], t_work);
        atomicAdd(&P.st->dbg[18], t_wait);
    }
    if (lane == 0 && wid == 1) {
        atomicAdd(&P.st->dbg[19], t_work);
        atomicAdd(&P.st->dbg[20], t_wait);
    }
#endif
#endif
    if (wid == 0 && lane < kExactTerms) s_tot[lane] = sum;
    __syncthreads();
}

__device__ void acc_candidate_exact(const KParams& P, double scale, int c, float* dyn) {
    if (c > P.NA) return;
#ifdef LO_PKO_STAMPS
    const unsigned long long c_t0 = __builtin_amdgcn_s_memtime();
#endif
    float* s_tot = dyn + kXcTotOff;                        // [kExactTerms]
    float* s_rec = s_tot + kExactTerms;                    // [kCandWords]
    const int tid = threadIdx.x;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = P.st->pose[k];
#ifdef LO_XC_PRIO
    // A/B build: the candidate's adder wave and its solving lane at the highest issue priority
    if (tid < kWave) __builtin_amdgcn_s_setprio(3);
#endif
    exact_sums_wg(P, T, scale, cand_delta(P, c), dyn, s_tot);
#ifdef LO_PKO_STAMPS
    if (tid == 0) atomicMax(&P.st->dbg[15], __builtin_amdgcn_s_memrealtime());   // the last candidate's sums end
#endif
    if (tid == 0) {
        float tot[kExactTerms], pn[12], delta[6];
#pragma unroll
        for (int k = 0; k < kExactTerms; ++k) tot[k] = s_tot[k];
#ifdef LO_PKO_STAMPS
        const unsigned long long sv0 = __builtin_amdgcn_s_memtime(), sr0 = __builtin_amdgcn_s_memrealtime();
#endif
        const bool conv = exact_solve_step(tot, T, P.tol_t, P.tol_r, pn, delta);
#ifdef LO_PKO_STAMPS
        if (c == 0) {                        // diagnostic: candidate 0's solve in shader cycles (dbg[8]) and in
            const float keep = pn[0] + delta[0];   // s_memrealtime ticks (dbg[9], 100 MHz): the launch's clock
            asm volatile("" :: "v"(keep));
            P.st->dbg[8] = __builtin_amdgcn_s_memtime() - sv0;
            P.st->dbg[9] = __builtin_amdgcn_s_memrealtime() - sr0;
        }
#ifndef LO_PKO_SUMS_COUNTERS
        {                                    // every candidate's solve: the largest (dbg[16]), the sum and count
            const float keep = pn[1] + delta[1];   // (dbg[17] / [18], cumulative) in shader cycles
            asm volatile("" :: "v"(keep));
            const unsigned long long cyc = __builtin_amdgcn_s_memtime() - sv0;
            atomicMax(&P.st->dbg[16], cyc);
            atomicAdd(&P.st->dbg[17], cyc);
            atomicAdd(&P.st->dbg[18], 1ull);
        }
        {                                    // the same solve again, now with its code in the instruction cache: the
            float tot2[kExactTerms], pn2[12], delta2[6];   // largest (dbg[19]) and the sum (dbg[20]) of its cycles
#pragma unroll
            for (int k = 0; k < kExactTerms; ++k) { tot2[k] = tot[k]; asm volatile("" : "+v"(tot2[k])); }
            const unsigned long long s2 = __builtin_amdgcn_s_memtime();
            const bool conv2 = exact_solve_step(tot2, T, P.tol_t, P.tol_r, pn2, delta2);
            const float keep = pn2[1] + delta2[1] + (conv2 ? 1.0f : 0.0f);
            asm volatile("" :: "v"(keep));
            const unsigned long long cyc = __builtin_amdgcn_s_memtime() - s2;
            atomicMax(&P.st->dbg[19], cyc);
            atomicAdd(&P.st->dbg[20], cyc);
        }
#endif
#endif
#pragma unroll
        for (int q = 0; q < 12; ++q) s_rec[q] = pn[q];
        s_rec[kCandCost] = tot[42];
        int k = 0;
        for (int r = 0; r < 6; ++r) for (int cc = r; cc < 6; ++cc) s_rec[kCandH + k++] = tot[r * 6 + cc];
#pragma unroll
        for (int j = 0; j < 6; ++j) { s_rec[kCandG + j] = tot[36 + j]; s_rec[kCandD + j] = delta[j]; }
        s_rec[kCandConv] = conv ? 1.0f : 0.0f;
        s_rec[kCandConv + 1] = 0.0f;
    }
    __syncthreads();
    if (tid < kCandWords) P.cand_rec[static_cast<size_t>(c) * kCandWords + tid] = s_rec[tid];
#ifdef LO_PKO_STAMPS
    if (tid == 0) {                          // diagnostic: candidate 0's cycles (dbg[7]); dbg[15] / [23]: the last
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // candidate's sums end / record end (s_memrealtime)
        if (c == 0) P.st->dbg[7] = __builtin_amdgcn_s_memtime() - c_t0;
        atomicMax(&P.st->dbg[23], __builtin_amdgcn_s_memrealtime());
    }
#endif
}

// Phase 1 of the PKO launch: correspondence count n_c, the exclusive rank -> block prefix of the per-block counts
// (s_pre, nb ints of LDS) and the normalisation scale -- iteration 0: std/6 of the accepted residuals from the
// per-block (count, sum, M2) by a Chan merge about the global mean (IterativeClosestPointOptimizer.cpp:304-316);
// later iterations: DevState::scale.  With nb <= 64 every block sits in wave 0, so the result does not depend on
// NW.  lead: this workgroup publishes the iteration-0 scale.
// The single-wave prefix's global loads (nb <= 64, wave 0, lane = block), issued by pko_body in the same round trip
// as the done flag instead of after it.
struct PrefixLoads {
    int c;
    double bs, bm, sc;
    uint64_t wm[kWavesPerBlock];
};

__device__ __forceinline__ void prefix_loads(const KParams& P, const ScanBufs& B, int it, PrefixLoads& pl) {
    const int lane = threadIdx.x & 63, nb = P.nb;
    const bool calc = it == 0 && !P.scale_given;
    pl.c = lane < nb ? B.blk_cnt[lane] : 0;
    pl.bs = (calc && lane < nb) ? 0.0 + P.blk_sum[lane] : 0.0;   // as `lsum += ...` from +0
    pl.bm = (calc && lane < nb) ? P.blk_m2[lane] : 0.0;
#pragma unroll
    for (int q = 0; q < kWavesPerBlock; ++q) {
        const int w = q * 64 + lane;
        pl.wm[q] = w < nb * kWavesPerBlock ? B.wmask[w] : 0;
    }
    pl.sc = calc ? 0.0 : B.st->scale;
}

template <int NW>
__device__ __forceinline__ void pko_prefix(const KParams& P, const ScanBufs& B, int it, bool lead, int* s_pre,
                                           int& nc_out, double& scale_out, uint64_t* s_wm = nullptr,
                                           const PrefixLoads* pre = nullptr) {
    constexpr int NT = NW * 64;
    DevState* st = B.st;
    __shared__ int s_iscan[NW];
    __shared__ double s_dscan[NW];
    __shared__ int s_nc;
    __shared__ double s_scale, s_mean;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const bool calc = it == 0 && !P.scale_given;           // iteration 0 computes the scale (unless it is given)
    if (P.direct_res) {
        if (tid == 0) { s_nc = P.n; s_scale = 1.0; }
        __syncthreads();
    } else if (P.nb <= 64) {
        // one wave, lane b = block b, one barrier: the same per-lane values and wave trees as the general path below
        // (with nb <= 64 every block sits in wave 0 there too), so the same bits.  s_wm (nullable): the blocks'
        // validity ballots prefetched into LDS for the sample phase.
        if (wid == 0) {
            const int nb = P.nb;
            PrefixLoads own;
            if (!pre) prefix_loads(P, B, it, own);
            const PrefixLoads& L = pre ? *pre : own;
            const int c = L.c;
            const double bs = L.bs, bm = L.bm;
            if (s_wm) {
#pragma unroll
                for (int q = 0; q < kWavesPerBlock; ++q) {
                    const int w = q * 64 + lane;
                    if (w < nb * kWavesPerBlock) s_wm[w] = L.wm[q];
                }
            }
            int inc = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) { const int t = __shfl_up(inc, o, 64); if (lane >= o) inc += t; }
            const int total = __shfl(inc, 63, 64);
            if (lane < nb) s_pre[lane] = inc - c;
            double scale;
            if (calc) {
                const double mean = total > 0 ? (0.0 + wave_total(bs)) / total : 0.0;
                double m2 = 0.0;
                if (c > 0) { const double dm = bs / c - mean; m2 = 0.0 + (bm + c * (dm * dm)); }
                const double M2 = 0.0 + wave_total(m2);
                const double var = total > 0 ? M2 / total : 0.0;
                scale = sqrt(var) / 6.0;                       // IterativeClosestPointOptimizer.cpp:314-315
            } else {
                scale = L.sc;
            }
            if (lane == 0) {
                s_nc = total;
                s_scale = scale;
                if (calc && lead) st->scale = scale;
            }
        }
        __syncthreads();
    } else {
        const int nb = P.nb;
        // (a) coalesced pass: block counts -> LDS, total count / residual sum
        int cnt = 0;
        double lsum = 0.0;
#pragma unroll 4
        for (int b = tid; b < nb; b += NT) {
            const int c = B.blk_cnt[b];
            s_pre[b] = c;
            cnt += c;
            if (calc) lsum += P.blk_sum[b];
        }
        cnt = wave_sum(cnt);
        lsum = wave_total(lsum);
        if (lane == 0) { s_iscan[wid] = cnt; s_dscan[wid] = lsum; }
        __syncthreads();
        if (tid == 0) {
            int run = 0;
            double tot = 0.0;
            for (int w = 0; w < NW; ++w) { run += s_iscan[w]; tot += s_dscan[w]; }
            s_nc = run;
            s_mean = run > 0 ? tot / run : 0.0;
        }
        __syncthreads();
        // (b) contiguous ranges of the counts (LDS) for the exclusive prefix; iteration 0: Chan merge of the
        //     per-block (count, sum, M2) about the global mean, coalesced
        const int per = (nb + NT - 1) / NT;
        const int b0 = min(tid * per, nb), b1 = min(b0 + per, nb);
        int loc = 0;
        for (int b = b0; b < b1; ++b) loc += s_pre[b];
        int inc = loc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) { const int t = __shfl_up(inc, o, 64); if (lane >= o) inc += t; }
        double m2 = 0.0;
        if (calc) {
            const double mean = s_mean;
#pragma unroll 4
            for (int b = tid; b < nb; b += NT) {
                const int c = s_pre[b];
                if (c > 0) { const double dm = P.blk_sum[b] / c - mean; m2 += P.blk_m2[b] + c * (dm * dm); }
            }
            m2 = wave_total(m2);
        }
        __syncthreads();                                         // s_iscan / s_dscan reuse
        if (lane == 63) s_iscan[wid] = inc;
        if (lane == 0) s_dscan[wid] = m2;
        __syncthreads();
        if (tid == 0) {
            int run = 0;
            double M2 = 0.0;
            for (int w = 0; w < NW; ++w) { const int c = s_iscan[w]; s_iscan[w] = run; run += c; M2 += s_dscan[w]; }
            if (calc) {
                const double var = s_nc > 0 ? M2 / s_nc : 0.0;
                s_scale = sqrt(var) / 6.0;                      // IterativeClosestPointOptimizer.cpp:314-315
                if (lead) st->scale = s_scale;
            } else {
                s_scale = st->scale;
            }
        }
        __syncthreads();
        int excl = s_iscan[wid] + inc - loc;
        for (int b = b0; b < b1; ++b) { const int c = s_pre[b]; s_pre[b] = excl; excl += c; }
        __syncthreads();
    }
    nc_out = s_nc;
    scale_out = s_scale;
}

// LDS of the PKO phases (one instance per workgroup).
template <int NW>
struct PkoLds {
    // p: the split EM's per-sample pdfs of each component (double-buffered), then the JS terms (>= 20 alphas)
    static constexpr int kPbuf = (2 * kMaxK * 64 * NW > 2000) ? 2 * kMaxK * 64 * NW : 2000;
    static constexpr int kJsPass = kPbuf / 100;
    double sd[kMaxS];
    double gmm[3 * kMaxK];
    double Pbin[100];
    double p[kPbuf];
    double dm[2 * kMaxK];
    double az[2 * kJsPass];
    int nan[kJsPass];                              // NaN terms per row of the current JS pass
    uint64_t wm[kWavesPerBlock * 64];              // ballots of <= 64 blocks, prefetched by the prefix
    int32_t draws[kMaxK];                          // k-means draws for S = P.S
};

// Phase 0: what later phases need but does not depend on n_c, so its latency hides behind the prefix phase: this
// thread's sample slot (s = tid) event-list bounds and base value for the three shuffle modes, the k-means draws for
// S = P.S, and (one alpha per workgroup) this alpha and Z.
struct PkoPrefetch {
    int lo[3], hi[3], base[3];
    double alpha, Z;
};
template <int NW>
__device__ __forceinline__ void pko_prefetch(const KParams& P, int wg, int G, PkoPrefetch& pf, PkoLds<NW>& L) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int m = 0; m < 3; ++m) { pf.lo[m] = 0; pf.hi[m] = 0; pf.base[m] = 0; }
    if (tid < P.S) {
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            pf.lo[m] = P.ev_off[m * (P.S + 1) + tid];
            pf.hi[m] = P.ev_off[m * (P.S + 1) + tid + 1];
            pf.base[m] = P.base[m * P.S + tid];
        }
    }
    const int D0 = P.K > 1 ? P.K - 1 : 1;
    if (tid < D0) L.draws[tid] = P.km_draws[P.S * D0 + tid];
    pf.alpha = 0.0;
    pf.Z = 0.0;
    if (G >= P.NA && 1 + wg <= P.NA) { pf.alpha = P.alphas[1 + wg]; pf.Z = P.Z[1 + wg]; }
}

// Phases 2-4 of the PKO for n_c >= 1 correspondences with normalisation scale `scale`: the reference's GMM sample,
// the GMM fit and this workgroup's slice of the JS grid (written to B.js).
template <int NW, bool ONE_WAVE>
__device__ __forceinline__ void pko_fit_js(const KParams& P, const ScanBufs& B, int wg, int G, int nc, double scale,
                                           const PkoPrefetch& pf, const int* s_pre, const uint64_t* s_wmask,
                                           PkoLds<NW>& L, unsigned long long* dbg) {
    constexpr int NT = NW * 64;
    DevState* st = B.st;
    const int tid = threadIdx.x;
    const bool lead = wg == 0;
    const bool one_alpha = G >= P.NA;                       // the single-scan launch: alpha 1 + wg only
    const double sden = (scale < 1e-6) ? 1e-6 : scale;     // std::max(scale, 1e-6)

    // ---- 2. the reference's GMM sample ----
    const int S = min(P.S, nc);
    for (int sidx = tid; sidx < S; sidx += NT) {
        int rank;
        if (sidx == tid && nc >= P.S && sidx < P.S) {          // prefetched bounds: one round of event loads
            const int mode = (nc <= 65535) ? ((nc & 1) ? 0 : 1) : 2;
            const int lo0 = mode == 0 ? pf.lo[0] : (mode == 1 ? pf.lo[1] : pf.lo[2]);
            const int hi0 = mode == 0 ? pf.hi[0] : (mode == 1 ? pf.hi[1] : pf.hi[2]);
            rank = mode == 0 ? pf.base[0] : (mode == 1 ? pf.base[1] : pf.base[2]);
            for (int e0 = lo0; e0 < hi0; e0 += 8) {             // ascending steps: the last one <= n - 1 wins
                int ev[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) ev[u] = (e0 + u < hi0) ? P.ev_steps[e0 + u] : 0x7fffffff;
#pragma unroll
                for (int u = 0; u < 8; ++u) if (ev[u] <= nc - 1) rank = ev[u];
            }
        } else {
            rank = pko_sample(P, nc, sidx);
        }
        LO_STAMP_WAIT(dbg, 13, sidx == 0);
        double v;
        if (P.direct_res) {
            v = P.direct_res[rank];
        } else {
            int lo = 0, hi = P.nb - 1;                          // last block with prefix <= rank
            while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (s_pre[mid] <= rank) lo = mid; else hi = mid - 1; }
            const int b = lo;
            // clamped: in-range for any data, so a workgroup that read a half-written state (a wave that saw the
            // lead's INSUFFICIENT flag after the others started) cannot index outside the block or loop long
            int k = min(max(rank - s_pre[b], 0), kBlock - 1);
            uint64_t m4[kWavesPerBlock];                        // the block's ballots: independent loads in flight
#pragma unroll
            for (int q = 0; q < kWavesPerBlock; ++q)
                m4[q] = s_wmask ? s_wmask[b * kWavesPerBlock + q] : B.wmask[b * kWavesPerBlock + q];
            int w = 0;
            uint64_t mk = m4[0];
#pragma unroll
            for (int q = 0; q + 1 < kWavesPerBlock; ++q) {
                const int c = __popcll(mk);
                if (w == q && k >= c) { k -= c; w = q + 1; mk = m4[q + 1]; }
            }
            // position of the k-th set bit of mk by halving windows (6 popcounts) instead of clearing k bits one
            // at a time (up to 63 dependent steps, the wave waits for its largest k); same bit
            int bit = 0;
#pragma unroll
            for (int wdt = 32; wdt >= 1; wdt >>= 1) {
                const int c = __popcll(mk & ((1ull << wdt) - 1));
                if (k >= c) { k -= c; mk >>= wdt; bit += wdt; }
            }
            bit = min(bit, kWave - 1);
            const int pidx = b * kBlock + w * kWave + bit;
            if (P.kd_res) {
                v = P.kd_res[pidx] / sden;                       // KDTree path: stored fp64 distance
            } else if (B.res) {
                v = B.res[pidx] / sden;                          // stored by the correspondence launch (same bits)
            } else {
                float T[12];
#pragma unroll
                for (int q = 0; q < 12; ++q) T[q] = B.pose_in ? B.pose_in[q] : st->pose[q];
                float wx, wy, wz;
                transform_pt(T, P.pts[3 * pidx], P.pts[3 * pidx + 1], P.pts[3 * pidx + 2], wx, wy, wz);
                v = residual_f64(P.tab[B.slot[pidx]], wx, wy, wz) / sden;   // :321-326
            }
        }
        LO_STAMP_WAIT(dbg, 14, sidx == 0);
        L.sd[sidx] = v;
    }
    __syncthreads();
    LO_STAMP(dbg, 2);

    // ---- 3. GMM ----
    const int D = P.K > 1 ? P.K - 1 : 1;
    const int32_t* draws = (S == P.S) ? L.draws : P.km_draws + S * D;
    if (ONE_WAVE) {                                             // wave 0 alone: see gmm_fit_1w
        switch (P.K) {
            case 1: gmm_fit_1w_dispatch<1>(L.sd, S, draws, L.gmm); break;
            case 2: gmm_fit_1w_dispatch<2>(L.sd, S, draws, L.gmm); break;
            default: gmm_fit_1w_dispatch<3>(L.sd, S, draws, L.gmm); break;
        }
    } else {
        unsigned long long* emst = lead ? P.em_stat : nullptr;
        switch (P.K) {                                          // every wave: see gmm_fit_split
            case 1: gmm_fit_dispatch<1>(L.sd, S, draws, L.gmm, L.p, L.dm, dbg, emst); break;
            case 2: gmm_fit_dispatch<2>(L.sd, S, draws, L.gmm, L.p, L.dm, dbg, emst); break;
            default: gmm_fit_dispatch<3>(L.sd, S, draws, L.gmm, L.p, L.dm, dbg, emst); break;
        }
    }
    __syncthreads();
    LO_STAMP(dbg, 12);
    if (lead && tid < 3 * P.K) st->gmm_out[tid] = L.gmm[tid];

    // ---- 4. JS divergence for this workgroup's alphas (calculate_js_divergence :710-787) ----
    // the EM's pdf buffers are dead now: they hold the terms of kJsPass alphas x 100 bins per pass (a single
    // workgroup per scan -- the batched launch -- needs 5 passes for the 100-alpha grid instead of 25).  The
    // pass's alphas and Z sit in LDS (L.az), loaded by the summing threads while the previous pass is summed, so
    // the term loop issues no global load and its iterations are independent chains the compiler interleaves.
    constexpr int kJsPass = PkoLds<NW>::kJsPass;
    constexpr int kTerms = kJsPass * 100;
    double* s_jsd = L.p;
    const int K = P.K;
    const double dr = P.trunc / 100.0;
    const int a_step = G * kJsPass;
    if (tid < kJsPass) L.nan[tid] = 0;                          // ordered by the barrier after the bins
    if (!one_alpha && tid < kJsPass) {
        const int ai = 1 + wg + tid * G;
        L.az[tid] = ai <= P.NA ? P.alphas[ai] : 0.0;
        L.az[kJsPass + tid] = ai <= P.NA ? P.Z[ai] : 0.0;
    }
    for (int b = tid; b < 100; b += NT) {
        const double r = dr * (1 + static_cast<double>(b));
        double g[kMaxK];                                         // independent pdf chains, then the ordered sum
#pragma unroll
        for (int m = 0; m < kMaxK; ++m) g[m] = m < K ? L.gmm[m] * gpdf(r, L.gmm[K + m], L.gmm[2 * K + m]) : 0.0;
        double Pr = 0.0;
#pragma unroll
        for (int m = 0; m < kMaxK; ++m) if (m < K) Pr += g[m];
        L.Pbin[b] = Pr + 1e-10;
    }
    __syncthreads();
    LO_STAMP(dbg, 10);
    for (int a0 = 1 + wg; a0 <= P.NA; a0 += a_step) {
        const int n_terms = one_alpha ? 100 : min(kJsPass, (P.NA - a0) / G + 1) * 100;   // this pass's alphas
#pragma unroll 4
        for (int q = 0; q < (kTerms + NT - 1) / NT; ++q) {
            const int idx = tid + q * NT;
            if (idx >= n_terms) break;
            const int a = idx / 100, b = idx - a * 100;
            const double alpha = one_alpha ? pf.alpha : L.az[a];
            const double pz = one_alpha ? pf.Z : L.az[kJsPass + a];
            const double r = dr * (1 + static_cast<double>(b));
            const double Pr = L.Pbin[b];
            const double Q = pko_kernel_w(r, alpha, P.pko_kernel) / (pz + 1e-10) + 1e-10;
            const double Mx = 0.5 * (Pr + Q);
            const double t = 0.5 * (Pr * log_pos(Pr / Mx) + Q * log_pos(Q / Mx));   // lo_math.h, <= 1 ulp from log
            // the reference skips NaN terms in its sum and count: the term is stored as +0 (adding +0 to the sum,
            // which starts at +0, is the same as skipping it) and counted here, so the sequential sum below is a
            // plain chain of adds
            const bool bad = isnan(t);
            if (bad) atomicAdd(&L.nan[a], 1);
            s_jsd[idx] = bad ? 0.0 : t;
        }
        __syncthreads();
        LO_STAMP(dbg, 11);
        if (tid < kJsPass) {
            const int ai = a0 + tid * G, an = ai + a_step;
            double nx_a = 0.0, nx_z = 0.0;                       // next pass's alpha and Z, in flight during the sum
            if (!one_alpha && an <= P.NA) { nx_a = P.alphas[an]; nx_z = P.Z[an]; }
            if (ai <= P.NA) {
                double cost = 0.0;                               // sequential, bin order (NaN terms are +0)
                const double cnt = static_cast<double>(100 - L.nan[tid]);
                const double* row = s_jsd + tid * 100;
                double vb[20], vn[20];                           // LDS reads of the next 20 bins in flight while
#pragma unroll                                                   // the serial adds consume the current ones
                for (int q = 0; q < 20; ++q) vb[q] = row[q];
                for (int b0 = 0; b0 < 100; b0 += 20) {
#pragma unroll
                    for (int q = 0; q < 20; ++q) vn[q] = (b0 + 20 < 100) ? row[b0 + 20 + q] : 0.0;
#pragma unroll
                    for (int q = 0; q < 20; ++q) cost += vb[q];
#pragma unroll
                    for (int q = 0; q < 20; ++q) vb[q] = vn[q];
                }
                B.js[ai] = cnt == 0.0 ? DBL_MAX : cost / cnt;
            }
            if (!one_alpha) { L.az[tid] = nx_a; L.az[kJsPass + tid] = nx_z; }
            L.nan[tid] = 0;                                      // read above; the next pass counts after the barrier
        }
        __syncthreads();
    }
    LO_STAMP(dbg, 6);
#ifdef LO_PKO_STAMPS
    if (dbg && tid == 0) dbg[22] = __builtin_amdgcn_s_memrealtime();   // the lead's JS end (100 MHz, chip-wide clock)
#endif
}

// wg / G: this workgroup's index among the G workgroups working on the scan (the JS alpha slices); in the
// single-scan launch, workgroups wg >= G are speculative normal-equation candidates (acc_candidate; XC: the
// reference-exact acc_candidate_exact, a separate instantiation so the default kernel's code is not touched).
// ONE_WAVE (batched launches of many scans): the GMM is fitted by wave 0 alone (gmm_fit_1w).
template <int NW, bool ONE_WAVE, bool XC = false>
__device__ __forceinline__ void pko_body(const KParams& P, const ScanBufs& B, int it, int wg, int G) {
    DevState* st = B.st;
    // the done flag, the single-wave prefix's loads and the prefetch below go out in one round trip; the flag is
    // tested once they are in flight (a converged scan leaves without writing anything)
    const int done0 = st->done || tail_gone(P);   // tail launch: scan already final (or the pipeline broken)
    PrefixLoads pl;
    const bool wave_prefix = !P.direct_res && P.nb <= 64;
    if (wave_prefix && threadIdx.x < 64) prefix_loads(P, B, it, pl);
    unsigned long long* dbg = nullptr;
#ifdef LO_PKO_STAMPS
    if (wg == 0) dbg = st->dbg;
    const unsigned long long t_launch = __builtin_amdgcn_s_memtime();   // dbg[0], stored by working launches only
    const unsigned long long rt_launch = __builtin_amdgcn_s_memrealtime();   // dbg[21] (chip-wide clock)
#endif
    // dynamic, nb ints: exclusive prefix of block counts (16-B aligned: the exact candidates read it with ds_read_b128,
    // and a misaligned 16-B LDS read is split -- the static part ends at a multiple of 8 only)
    extern __shared__ __attribute__((aligned(16))) int s_pre[];
    __shared__ PkoLds<NW> L;
    PkoPrefetch pf;
    pko_prefetch<NW>(P, wg, G, pf, L);
    if (done0) return;

    const int tid = threadIdx.x;
    const bool lead = wg == 0;
    if constexpr (NW == 4 && !ONE_WAVE && XC) {
        // reference-exact candidates need only the scale, which is given (iteration 0: k_exact_scale's, before this
        // launch): they start their sums at once instead of after the prefix phase (~4k cycles).  Not in a tail launch,
        // whose workgroups must see the scan still pending after the prefix (below) before they write anything.
        if (wg >= G && P.scale_given && !P.tail) {
            acc_candidate_exact(P, st->scale, wg - G, reinterpret_cast<float*>(s_pre));
            return;
        }
    }
    // ---- 1. n_c, rank -> block prefix, iteration-0 scale ----
    int nc;
    double s_scale;
    const uint64_t* s_wmask = P.nb <= 64 && !P.direct_res ? L.wm : nullptr;
    pko_prefix<NW>(P, B, it, lead, s_pre, nc, s_scale, L.wm, &pl);   // pl is set where it is read (nb <= 64)
    if (P.tail) {
        // A tail launch tests the scan's state once more before acting on what the prefix read: another workgroup of
        // this launch may have published the scan final (too few correspondences) after this one passed done0, and
        // the context stream may already run the next scan on the same buffers.  fin is published before the next
        // scan can start, so a workgroup that still sees it unpublished here read this scan's data.
        __shared__ int s_gone;
        if (tid == 0) s_gone = tail_gone(P) ? 1 : 0;
        __syncthreads();
        if (s_gone) return;
    }
    if (!P.direct_res && nc < P.min_corr) {                     // :298-302
        if (lead && tid == 0) { st->status = LO_INSUFFICIENT; st->done = 1; st->n_corr = nc; publish_final(P); }
        return;
    }
    if constexpr (NW == 4 && !ONE_WAVE) {
        if (wg >= G) {                                          // after the scale: the candidates need it
            if constexpr (XC) acc_candidate_exact(P, s_scale, wg - G, reinterpret_cast<float*>(s_pre));
            else acc_candidate(P, s_scale, wg - G);
            return;
        }
    }
    if (lead && tid == 0) st->n_corr = nc;
    if (!P.use_pko || nc == 0) return;                          // consumers use robust_loss_delta / 1.0
#ifdef LO_PKO_STAMPS
    if (dbg && tid == 0) { dbg[0] = t_launch; dbg[21] = rt_launch; }
#endif
    LO_STAMP(dbg, 1);
    pko_fit_js<NW, ONE_WAVE>(P, B, wg, G, nc, s_scale, pf, s_pre, s_wmask, L, dbg);
}

}  // namespace lo
