// lo_seqsum.h — the reference's SEQUENTIAL floating-point sums, reproduced bit for bit by a whole workgroup.
//
// The reference forms its iteration-0 normalisation scale (IterativeClosestPointOptimizer.cpp:304-316) as
// std::accumulate over the sorted residuals, then a second loop over (r - mean)^2: two chains of ~n dependent fp64
// adds (~8 cycles each on one lane).  Both sums add NON-NEGATIVE terms, so the running sum s never decreases, and
// while s stays inside one binade [2^E, 2^(E+1)) every partial sum is a multiple of u = ulp(2^E):
//     fl(s + x) = s + u * rint(x / u)                       (exact; x / u is a power-of-two scaling)
// unless x / u is exactly halfway between two integers (round-half-even then depends on s's last bit) or the result
// leaves the binade.  So a run of steps inside one binade is an INTEGER prefix sum -- associative, parallel.
//
// mono_seq_sum (one workgroup of NT threads, PT consecutive terms per thread):
//   1. an approximate prefix sum T_j (fp64, tree order) predicts each step's binade e_j = ilogb(T_j);
//   2. "heads" split the terms into segments of constant predicted binade: the first non-zero term, every term whose
//      predicted binade differs from its predecessor's, every halfway term; every other term contributes
//      q_j = rint(x_j / u_j) to an int64 prefix sum P (block scan);
//   3. one wave walks the heads in order: a head's step is done directly (s = fl(s + x_h)); the rest of its segment
//      [h + 1, next head) is accepted as s + u * (P_end - P_h) when s really lies in the predicted binade and the
//      result stays one ulp inside it (then every step of the segment rounded exactly as claimed: each exact partial sum
//      lies in the binade, none is a tie), otherwise that segment is summed term by term (rare: T_j and s_j straddle a
//      power of two).
// The result is the sequential sum's exact bits for any input: the prediction only decides how much work is parallel.
// ~30-70 heads for a KITTI scan's residuals; 4k terms cost two block scans and a 50-step walk instead of a 4k-step
// chain.  Prototype + randomized check against the sequential loop: tests/test_seqsum.py (CPU) and
// tests/test_gpu_exact.py (bit-identical scales through the whole GN step).
#pragma once
#include <climits>

#include "lo_device.h"

namespace lo {

constexpr int kSeqThreads = 1024;              // workgroup of the scale kernels
constexpr int kSeqWaves = kSeqThreads / kWave;
constexpr int kSeqHeadCap = 1024;              // heads per pass (more: the pass falls back to the plain chain)
constexpr int kExpNone = -100000;              // "binade" of a zero / subnormal / non-positive prediction

__device__ __forceinline__ int binade64(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const int f = static_cast<int>((b >> 52) & 0x7FF);
    return (v > 0.0 && f != 0 && f != 0x7FF) ? f - 1023 : kExpNone;
}

__device__ __forceinline__ double rl64d(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ long long rl64i(long long v, int l) {
    const uint64_t u = static_cast<uint64_t>(v);
    const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(u)), l));
    const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(u >> 32)), l));
    return static_cast<long long>((static_cast<uint64_t>(hi) << 32) | lo);
}

// Exclusive prefix over the workgroup of one value per thread (wave scan by shuffles, wave totals through LDS), and
// the total.  s_w: kSeqWaves entries, free again when the function returns.
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* s_w, T& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    T inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    T ex = __shfl_up(inc, 1, 64);
    if (lane == 0) ex = T(0);
    if (lane == 63) s_w[wid] = inc;
    __syncthreads();
    T before = T(0), tot = T(0);
#pragma unroll
    for (int w = 0; w < kSeqWaves; ++w) {
        const T x = s_w[w];
        if (w < wid) before += x;
        tot += x;
    }
    __syncthreads();
    total = tot;
    return before + ex;
}

// Maximum over the workgroup of one value per thread (s_w: kSeqWaves entries, free again on return).
__device__ __forceinline__ double block_max(double v, double* s_w) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { const double t = __shfl_xor(v, o, 64); v = t > v ? t : v; }
    if (lane == 0) s_w[wid] = v;
    __syncthreads();
    double m = s_w[0];
#pragma unroll
    for (int w = 1; w < kSeqWaves; ++w) m = s_w[w] > m ? s_w[w] : m;
    __syncthreads();
    return m;
}

struct SeqScratch {
    double wd[kSeqWaves];
    long long wl[kSeqWaves];
    int wi[kSeqWaves];
    int elast[kSeqThreads];
    int h_idx[kSeqHeadCap];
    int h_e[kSeqHeadCap];
    long long h_p[kSeqHeadCap];
    double result;
    int e_carry;
    int nheads, fb_seg, fb_terms;              // walk statistics (heads; segments / terms summed term by term)
};

// s_in + x_0 + x_1 + ... + x_{cnt-1}, each addition rounded separately in index order, for x_j >= +0 (non-negative,
// no NaN; +inf is never among the first cnt terms), the terms in s_x[0, cnt) (LDS); thread t works on terms
// t*PT .. t*PT + PT - 1.  Carry-in for chunked use: T0 = the approximate prefix before term 0, e0 = the predicted binade
// of the term before term 0, head0 = term 0 starts a segment whatever its binade.  Every thread returns the sum;
// S.e_carry receives the predicted binade of the last term.  Returns false (nothing computed) when a pass has more
// than kSeqHeadCap heads.  The per-term quantities are recomputed in each pass instead of being kept in arrays (the
// arrays spilled to scratch at PT >= 8).
template <int PT>
__device__ __forceinline__ bool mono_seq_sum(int cnt, const double* s_x, SeqScratch& S, double T0, int e0, bool head0, double s_in,
                             double& s_out) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int base = tid * PT;
    auto term = [&](int a) { return base + a < cnt ? s_x[base + a] : 0.0; };
    // 1. approximate prefix: this thread's total, the workgroup scan, the last term's predicted binade
    double run = 0.0;
#pragma unroll
    for (int a = 0; a < PT; ++a) run += term(a);
    double ttot;
    const double tex = T0 + block_excl_scan<double>(run, S.wd, ttot);
    S.elast[tid] = binade64(tex + run);
    __syncthreads();
    const int e_in = tid ? S.elast[tid - 1] : e0;
    // 2. heads and integer steps (one pass counts them, the next files them; both recompute the same values)
    auto classify = [&](int a, double tl, int ep, int& E, long long& qa) -> bool {
        const int j = base + a;
        const double xv = term(a);
        E = binade64(tex + tl);
        qa = 0;
        if (!(j < cnt && (xv != 0.0 || (head0 && j == 0)))) return false;   // a chunk's first term heads it even when zero
        if (E < -1000 || E != ep || (head0 && j == 0)) return true;
        const double t = ldexp(xv, 52 - E);                                // exact power-of-two scaling
        const double f = floor(t), fr = t - f;                             // exact (t < 2^54)
        if (fr == 0.5) return true;                                        // halfway: depends on s's last bit
        qa = static_cast<long long>(f) + (fr > 0.5 ? 1 : 0);
        return false;
    };
    long long ql = 0;
    int nhl = 0;
    {
        double tl = 0.0;
        int ep = e_in;
#pragma unroll
        for (int a = 0; a < PT; ++a) {
            tl += term(a);
            int E;
            long long qa;
            nhl += classify(a, tl, ep, E, qa) ? 1 : 0;
            ql += qa;
            ep = E;
        }
    }
    long long ptot;
    const long long pex = block_excl_scan<long long>(ql, S.wl, ptot);
    int htot;
    const int hbase = block_excl_scan<int>(nhl, S.wi, htot);
    if (htot > kSeqHeadCap) return false;                       // uniform: every thread sees htot
    {
        double tl = 0.0;
        int ep = e_in, hk = hbase;
        long long prun = pex;
#pragma unroll
        for (int a = 0; a < PT; ++a) {
            tl += term(a);
            int E;
            long long qa;
            const bool hd = classify(a, tl, ep, E, qa);
            prun += qa;
            if (hd) { S.h_idx[hk] = base + a; S.h_e[hk] = E; S.h_p[hk] = prun; ++hk; }
            ep = E;
        }
        if (tid == kSeqThreads - 1) S.e_carry = ep;
    }
    if (tid == 0) S.nheads = htot;
    __syncthreads();
    // 3. the walk (wave 0, wave-uniform): lane l of a 64-head window holds head k0 + l and precomputes what the
    //    sequential step needs -- the head's term, the segment's sum u * Q, the binade floor 2^E and the largest
    //    result the segment may reach (2^(E+1) - u); a one-term segment, or a lane past the last head, passes any
    //    check (its dq is 0), a segment without a valid binade fails every check.  Heads go eight at a time as a
    //    branch-free chain of two adds each; a group in which any check failed is redone head by head from its start
    if (wid == 0) {
        double s = s_in;
        int fbs = 0, fbt = 0;
        for (int k0 = 0; k0 < htot; k0 += 64) {
            const int kk = k0 + lane;
            int hi = 0, hend = cnt;
            double hx = -0.0, dq = -0.0, lo_e = -__builtin_inf(), top = __builtin_inf();   // x + -0 == x, also for x = -0
            if (kk < htot) {
                hi = S.h_idx[kk];
                const int E = S.h_e[kk];
                const long long hp = S.h_p[kk];
                long long pend = ptot;
                hx = s_x[hi];
                if (kk + 1 < htot) { pend = S.h_p[kk + 1]; hend = S.h_idx[kk + 1]; }
                const long long Q = pend - hp;
                if (hend > hi + 1) {
                    lo_e = __builtin_inf();
                    top = 0.0;
                    if (E >= -1000 && Q >= 0 && Q < (1ll << 53)) {
                        const double u = ldexp(1.0, E - 52);
                        dq = static_cast<double>(Q) * u;
                        lo_e = ldexp(1.0, E);
                        top = ldexp(1.0, E + 1) - u;
                    }
                }
            }
            const int m = min(64, htot - k0);
            for (int l0 = 0; l0 < m; l0 += 8) {
                const double s0 = s;
                int bad = 0;
#pragma unroll
                for (int u = 0; u < 8; ++u) {                    // lanes past m are the no-op heads above
                    const double s1 = s + rl64d(hx, l0 + u);     // the head's own step, as the reference does it
                    const double R = s1 + rl64d(dq, l0 + u);     // exact when the segment stays in the binade
                    bad |= (s1 >= rl64d(lo_e, l0 + u) && R <= rl64d(top, l0 + u)) ? 0 : 1;
                    s = R;
                }
                if (__builtin_amdgcn_readfirstlane(bad)) {       // uniform: redo the group head by head
                    s = s0;
                    for (int l = l0; l < min(l0 + 8, m); ++l) {
                        const int h = __builtin_amdgcn_readlane(hi, l), end = __builtin_amdgcn_readlane(hend, l);
                        s = s + rl64d(hx, l);
                        const double R = s + rl64d(dq, l);
                        if (__builtin_amdgcn_readfirstlane((s >= rl64d(lo_e, l) && R <= rl64d(top, l)) ? 1 : 0)) {
                            s = R;
                        } else {
                            for (int j = h + 1; j < end; ++j) s = s + s_x[j];
                            ++fbs;
                            fbt += end - h - 1;
                        }
                    }
                }
            }
        }
        if (lane == 0) { S.result = s; S.fb_seg = fbs; S.fb_terms = fbt; }
    }
    __syncthreads();
    s_out = S.result;
    return true;
}

// The plain chain (fallback): wave 0 adds s_x[0, cnt) to s in order, one rounding per term; every thread returns it.
__device__ inline double chain_seq_sum(const double* s_x, int cnt, double s, SeqScratch& S) {
    if ((threadIdx.x >> 6) == 0) {
        for (int j = 0; j < cnt; ++j) s = s + s_x[j];
        if (threadIdx.x == 0) S.result = s;
    }
    __syncthreads();
    return S.result;
}

}  // namespace lo

namespace lo {

// ---------------------------------------------------------------------------------------------------------------------
// Signed fp32 sequential sums (the reference's build_ne accumulates H, g and the cost as running fp32 sums,
// IterativeClosestPointOptimizer.cpp:359-415).  The same idea as mono_seq_sum, for terms of either sign: while the
// running sum s keeps its sign and binade [2^E, 2^(E+1)) in magnitude, fl(s + x) = s + u rint(x / u), u = 2^(E-23).
// The partial sums of a segment are no longer monotone, so the prediction carries the proof: a term heads a segment
// also when its predicted prefix T lies within M = 2^(E-9) of either edge of its binade.  Inside a segment every T_j
// is then at least M from the edges, and the true partial sums differ from T_j by at most |s_h - T_h| (known once the
// walk reaches the head) + (end - h) u / 2 (one half-ulp per step) + the fp64 error of T (< 2^(E-30)): when that total
// stays below M - u, every partial sum of the segment is inside the binade, one ulp from its edges, and the integer
// model is exact for each step.  The fp64 error of T is bounded per chunk by 2^-46 times the largest magnitude any of its
// partial sums reaches (fewer than 64 roundings per predicted term), so a chunk whose sums cancel large values only
// loses parallelism, never exactness.  Terms come in chunks (kSeqThreads * PT), each chunk starting a segment, with
// the exact running sum carried in as the next chunk's prediction base.
// ---------------------------------------------------------------------------------------------------------------------
constexpr int kSHeadCap = 4096;

struct SeqScratchS {
    double wd[kSeqWaves];
    long long wl[kSeqWaves];
    int wi[kSeqWaves];
    int elast[kSeqThreads];
    int glast[kSeqThreads];
    int h_idx[kSHeadCap];
    int h_e[kSHeadCap];
    long long h_p[kSHeadCap];
    double h_t[kSHeadCap];
    float result;
    int e_carry, g_carry;
    int nheads, fb_seg;
};

__device__ __forceinline__ int binade_abs(double v) {       // binade of |v| when it is a normal fp32 magnitude
    const double a = fabs(v);
    const uint64_t b = __builtin_bit_cast(uint64_t, a);
    const int f = static_cast<int>((b >> 52) & 0x7FF);
    const int e = f - 1023;
    return (a > 0.0 && f != 0x7FF && e >= -120 && e <= 126) ? e : kExpNone;
}

// s_in + x_0 + ... + x_{cnt-1} in fp32, one rounding per addition in index order; thread t holds terms t*PT.. (zeros past
// cnt), s_x[0, cnt) the same terms (LDS).  T0 / e0 / g0: the prediction base, binade and sign carried in from the
// previous chunk; term 0 always starts a segment.  Every thread returns the sum and the carries; false (nothing
// computed) when the chunk has more than kSHeadCap heads.
template <int PT>
__device__ __forceinline__ bool signed_seq_sum(int cnt, const float* s_x, SeqScratchS& S, double T0, int e0, int g0, float s_in,
                               float& s_out, int& e_out, int& g_out) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int base = tid * PT;
    auto term = [&](int a) { return base + a < cnt ? s_x[base + a] : 0.0f; };
    double run = 0.0, amax = fabs(T0);
#pragma unroll
    for (int a = 0; a < PT; ++a) {
        run += static_cast<double>(term(a));
        amax = fmax(amax, fabs(run));
    }
    double ttot;
    const double tex = T0 + block_excl_scan<double>(run, S.wd, ttot);
    {
        const double Tl = tex + run;
        S.elast[tid] = binade_abs(Tl);
        S.glast[tid] = Tl > 0.0 ? 1 : (Tl < 0.0 ? -1 : 0);
    }
    __syncthreads();
    const int e_in = tid ? S.elast[tid - 1] : e0, g_in = tid ? S.glast[tid - 1] : g0;
    // predicted binade / sign of term a's prefix, whether it lies within M of its binade's edges, and its step
    auto classify = [&](int a, double T, int ep, int gp, int& E, int& G, long long& qa) -> bool {
        const int j = base + a;
        const float xv = term(a);
        E = binade_abs(T);
        G = T > 0.0 ? 1 : (T < 0.0 ? -1 : 0);
        qa = 0;
        if (!(j < cnt && (xv != 0.0f || j == 0))) return false;          // a chunk's first term heads it even when zero
        const double at = fabs(T), M = ldexp(1.0, E - 9);
        const bool edge = E == kExpNone || at < ldexp(1.0, E) + M || at > ldexp(1.0, E + 1) - M;
        if (edge || E != ep || G != gp || j == 0) return true;
        const double t = ldexp(static_cast<double>(xv), 23 - E);         // exact
        const double f = floor(t), fr = t - f;
        if (fr == 0.5) return true;
        qa = static_cast<long long>(f) + (fr > 0.5 ? 1 : 0);
        return false;
    };
    long long ql = 0;
    int nhl = 0;
    {
        double tl = 0.0;
        int ep = e_in, gp = g_in;
#pragma unroll
        for (int a = 0; a < PT; ++a) {
            tl += static_cast<double>(term(a));
            const double T = tex + tl;
            amax = fmax(amax, fabs(T));
            int E, G;
            long long qa;
            nhl += classify(a, T, ep, gp, E, G, qa) ? 1 : 0;
            ql += qa;
            ep = E;
            gp = G;
        }
    }
    amax = fmax(amax, fabs(tex));
    long long ptot;
    const long long pex = block_excl_scan<long long>(ql, S.wl, ptot);
    int htot;
    const int hbase = block_excl_scan<int>(nhl, S.wi, htot);
    if (htot > kSHeadCap) return false;
    const double eps_t = ldexp(block_max(amax, S.wd), -46);    // bound on |T_j - exact prefix| for every term
    {
        double tl = 0.0;
        int ep = e_in, gp = g_in, hk = hbase;
        long long prun = pex;
#pragma unroll
        for (int a = 0; a < PT; ++a) {
            tl += static_cast<double>(term(a));
            const double T = tex + tl;
            int E, G;
            long long qa;
            const bool hd = classify(a, T, ep, gp, E, G, qa);
            prun += qa;
            if (hd) { S.h_idx[hk] = base + a; S.h_e[hk] = E; S.h_p[hk] = prun; S.h_t[hk] = T; ++hk; }
            ep = E;
            gp = G;
        }
        if (tid == kSeqThreads - 1) { S.e_carry = ep; S.g_carry = gp; }
    }
    if (tid == 0) S.nheads = htot;
    __syncthreads();
    if (wid == 0) {
        // lane l of a 64-head window precomputes head k0 + l's checks: the binade [2^E, 2^(E+1)), the allowed distance
        // of the head's result from its prediction (M - the segment's rounding and T error budget), the segment's sum;
        // a one-term segment or a lane past the last head passes (dq 0), a segment without a binade fails.  Eight heads
        // at a time as a branch-free chain; a group with a failed check is redone head by head from its start
        float s = s_in;
        int fbs = 0;
        for (int k0 = 0; k0 < htot; k0 += 64) {
            const int kk = k0 + lane;
            int hi = 0, hend = cnt, hg = 0, pass = 1;
            double ht = 0.0, lo_e = __builtin_inf(), maxdev = -1.0, dq = -0.0;          // x + -0 == x, also for x = -0
            float hx = -0.0f;
            if (kk < htot) {
                hi = S.h_idx[kk];
                const int E = S.h_e[kk];
                const long long hp = S.h_p[kk];
                long long pend = ptot;
                ht = S.h_t[kk];
                hx = s_x[hi];
                if (kk + 1 < htot) { pend = S.h_p[kk + 1]; hend = S.h_idx[kk + 1]; }
                pass = hend > hi + 1 ? 0 : 1;
                if (!pass && E != kExpNone) {
                    const double u = ldexp(1.0, E - 23);
                    lo_e = ldexp(1.0, E);
                    hg = ht > 0.0 ? 1 : -1;
                    maxdev = ldexp(1.0, E - 9) - (static_cast<double>(hend - hi) * 0.5 + 1.0) * u - 2.0 * eps_t;
                    dq = static_cast<double>(pend - hp) * u;
                }
            }
            auto check = [&](double d, int l) -> bool {
                const double ad = fabs(d), le = rl64d(lo_e, l);
                const bool sgn = __builtin_amdgcn_readlane(hg, l) > 0 ? d > 0.0 : d < 0.0;
                return __builtin_amdgcn_readlane(pass, l) != 0 ||
                       (ad >= le && ad < 2.0 * le && sgn && fabs(d - rl64d(ht, l)) <= rl64d(maxdev, l));
            };
            auto rlf = [](float v, int l) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l)); };
            const int m = min(64, htot - k0);
            for (int l0 = 0; l0 < m; l0 += 8) {
                const float s0 = s;
                int bad = 0;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    s = s + rlf(hx, l0 + u);
                    const double d = static_cast<double>(s);
                    bad |= check(d, l0 + u) ? 0 : 1;
                    s = static_cast<float>(d + rl64d(dq, l0 + u));
                }
                if (__builtin_amdgcn_readfirstlane(bad)) {
                    s = s0;
                    for (int l = l0; l < min(l0 + 8, m); ++l) {
                        const int h = __builtin_amdgcn_readlane(hi, l), end = __builtin_amdgcn_readlane(hend, l);
                        s = s + rlf(hx, l);
                        const double d = static_cast<double>(s);
                        if (__builtin_amdgcn_readfirstlane(check(d, l) ? 1 : 0)) {
                            s = static_cast<float>(d + rl64d(dq, l));
                        } else {
                            for (int j = h + 1; j < end; ++j) s = s + s_x[j];
                            ++fbs;
                        }
                    }
                }
            }
        }
        if (lane == 0) { S.result = s; S.fb_seg = fbs; }
    }
    __syncthreads();
    s_out = S.result;
    e_out = S.e_carry;
    g_out = S.g_carry;
    return true;
}

}  // namespace lo
