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

// Exclusive prefix over the workgroup (NT threads) of one value per thread (wave scan by shuffles, wave totals through
// LDS), and the total.  s_w: NT / 64 entries, free again when the function returns.
template <typename T, int NT = kSeqThreads>
__device__ __forceinline__ T block_excl_scan(T v, T* s_w, T& total) {
    constexpr int kNW = NT / kWave;
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
    for (int w = 0; w < kNW; ++w) {
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
    double2 xd[kWave];                         // the walk's window of (head term, segment sum), read as broadcasts
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
    // 3. the walk (wave 0, wave-uniform): lane l of a 64-head window holds head k0 + l and precomputes the head's
    //    term, the segment's sum u * Q and the interval the sum right after the head's step must lie in for the
    //    segment to stay in its binade, [2^E, 2^(E+1) - u - u * Q] (a one-term segment or a lane past the last head:
    //    any sum; a segment without a valid binade: none).  The 64 heads run as a plain chain of two adds each, the
    //    operands broadcast from LDS, lane l keeping the sum after head l's step; the checks then run lane-parallel,
    //    and from a failed check on the window goes head by head (that head's sum is exact: the earlier ones passed)
    if (wid == 0) {
        double s = s_in;
        int fbs = 0, fbt = 0;
        for (int k0 = 0; k0 < htot; k0 += 64) {
            const int kk = k0 + lane;
            int hi = 0, hend = cnt;
            double hx = -0.0, dq = -0.0, dlo = -__builtin_inf(), dhi = __builtin_inf();   // x + -0 == x, also for x = -0
            if (kk < htot) {
                hi = S.h_idx[kk];
                const int E = S.h_e[kk];
                const long long hp = S.h_p[kk];
                long long pend = ptot;
                hx = s_x[hi];
                if (kk + 1 < htot) { pend = S.h_p[kk + 1]; hend = S.h_idx[kk + 1]; }
                const long long Q = pend - hp;
                if (hend > hi + 1) {
                    dlo = __builtin_inf();
                    dhi = -__builtin_inf();
                    if (E >= -1000 && Q >= 0 && Q < (1ll << 53)) {
                        const double u = ldexp(1.0, E - 52);
                        dq = static_cast<double>(Q) * u;
                        dlo = ldexp(1.0, E);
                        dhi = (ldexp(1.0, E + 1) - u) - dq;      // exact: multiples of u below 2^(E+1)
                    }
                }
            }
            S.xd[lane] = make_double2(hx, dq);
            double rec = 0.0;
#pragma unroll
            for (int l = 0; l < 64; ++l) {                       // lanes past the window are no-op heads
                const double2 v = S.xd[l];
                s = s + v.x;                                     // the head's own step, as the reference does it
                rec = lane == l ? s : rec;
                s = s + v.y;                                     // exact when the segment stays in the binade
            }
            const unsigned long long badm = __ballot(!(rec >= dlo && rec <= dhi));
            if (badm) {                                          // uniform
                const int m = min(64, htot - k0), f = __builtin_ctzll(badm);
                s = rl64d(rec, f);
                {
                    const int h = __builtin_amdgcn_readlane(hi, f), end = __builtin_amdgcn_readlane(hend, f);
                    for (int j = h + 1; j < end; ++j) s = s + s_x[j];
                    ++fbs;
                    fbt += end - h - 1;
                }
                for (int l = f + 1; l < m; ++l) {
                    const int h = __builtin_amdgcn_readlane(hi, l), end = __builtin_amdgcn_readlane(hend, l);
                    s = s + rl64d(hx, l);
                    if (__builtin_amdgcn_readfirstlane((s >= rl64d(dlo, l) && s <= rl64d(dhi, l)) ? 1 : 0)) {
                        s = s + rl64d(dq, l);
                    } else {
                        for (int j = h + 1; j < end; ++j) s = s + s_x[j];
                        ++fbs;
                        fbt += end - h - 1;
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

// ---------------------------------------------------------------------------------------------------------------------
// Halfway ties without heads: the two-state form of a segment.
// Inside binade E the running sum is s = Q u (u = 2^(E-52), Q in [2^52, 2^53)).  A term x with t = x / u adds
// rint(t) to Q -- unless t is halfway (t = f + 1/2), where round-half-even gives Q + f when Q + f is even and
// Q + f + 1 otherwise: the step depends on Q's parity and always leaves Q even.  So every step is a map on the
// parity p = Q & 1 with an integer increment, Q -> Q + d_p, p -> p'_p, and a run of steps composes into one such map
// (SeqTx) -- associative, so a segment's whole effect is a (segmented) scan, and ties no longer split segments.  The
// walk then only stops where the running sum crosses a power of two or comes close to one (mono_sum_tx below): a
// KITTI scan's ~200 tie heads drop to ~25.
// ---------------------------------------------------------------------------------------------------------------------
struct SeqTx {
    long long d0, d1;        // Q increment for entry parity 0 / 1
    int p;                   // bit q: the exit parity for entry parity q
};
constexpr long long kTxSat = 1ll << 61;        // saturated increment (never exact: fails every check)
__device__ __forceinline__ SeqTx tx_ident() { return SeqTx{0, 0, 2}; }
__device__ __forceinline__ SeqTx tx_then(const SeqTx& a, const SeqTx& b) {   // a, then b
    const int a0 = a.p & 1, a1 = (a.p >> 1) & 1;
    const long long e0 = a.d0 + (a0 ? b.d1 : b.d0);
    const long long e1 = a.d1 + (a1 ? b.d1 : b.d0);
    return SeqTx{e0 < kTxSat ? e0 : kTxSat, e1 < kTxSat ? e1 : kTxSat, ((b.p >> a0) & 1) | (((b.p >> a1) & 1) << 1)};
}
// One term's step on binade E appended to m (x >= +0, t = x / u < 2^53: the caller's head rule guarantees it):
// t = f + r exactly; a halfway r rounds Q + f to even, otherwise Q gains rint(t).
__device__ __forceinline__ void tx_push(SeqTx& m, double x, int E) {
    const double t = ldexp(x, 52 - E);
    const double f = floor(t), fr = t - f;
    const long long fi = static_cast<long long>(f);
    const int fb = static_cast<int>(fi & 1), p0 = m.p & 1, p1 = (m.p >> 1) & 1;
    if (fr == 0.5) {
        m.d0 += fi + (p0 ^ fb);
        m.d1 += fi + (p1 ^ fb);
        m.p = 0;
    } else {
        const long long q = fi + (fr > 0.5 ? 1 : 0);
        const int b = static_cast<int>(q & 1);
        m.d0 += q;
        m.d1 += q;
        m.p = (p0 ^ b) | ((p1 ^ b) << 1);
    }
}

// Wave-wide inclusive scan of a POD of 32-bit words by DPP (row_shr 1/2/4/8, then row_bcast 15/31 into the upper
// rows): the earlier lane's value is combined in front, op(earlier, later).  Lanes without a source keep `ident`.
template <int N> struct Words { int w[N]; };
template <int CTRL, int RM, typename T>
__device__ __forceinline__ T dpp_pod(const T& v, const T& old) {
    static_assert(sizeof(T) % 4 == 0, "32-bit words");
    constexpr int N = sizeof(T) / 4;
    const Words<N> a = __builtin_bit_cast(Words<N>, v), o = __builtin_bit_cast(Words<N>, old);
    Words<N> r;
#pragma unroll
    for (int i = 0; i < N; ++i) r.w[i] = __builtin_amdgcn_update_dpp(o.w[i], a.w[i], CTRL, RM, 0xf, false);
    return __builtin_bit_cast(T, r);
}
template <typename T, typename Op>
__device__ __forceinline__ T wave_incl_scan(T v, const T& ident, Op op) {
    v = op(dpp_pod<0x111, 0xf>(v, ident), v);       // row_shr:1
    v = op(dpp_pod<0x112, 0xf>(v, ident), v);       // row_shr:2
    v = op(dpp_pod<0x114, 0xf>(v, ident), v);       // row_shr:4
    v = op(dpp_pod<0x118, 0xf>(v, ident), v);       // row_shr:8   (16-lane rows scanned)
    v = op(dpp_pod<0x142, 0xa>(v, ident), v);       // row_bcast:15 into rows 1, 3
    v = op(dpp_pod<0x143, 0xc>(v, ident), v);       // row_bcast:31 into rows 2, 3
    return v;
}
template <typename T>
__device__ __forceinline__ T readlane_pod(const T& v, int l) {
    constexpr int N = sizeof(T) / 4;
    Words<N> a = __builtin_bit_cast(Words<N>, v);
#pragma unroll
    for (int i = 0; i < N; ++i) a.w[i] = __builtin_amdgcn_readlane(a.w[i], l);
    return __builtin_bit_cast(T, a);
}
template <typename T>
__device__ __forceinline__ T shfl_up1_pod(const T& v, const T& ident) {
    constexpr int N = sizeof(T) / 4;
    const Words<N> a = __builtin_bit_cast(Words<N>, v);
    Words<N> r;
#pragma unroll
    for (int i = 0; i < N; ++i) r.w[i] = __shfl_up(a.w[i], 1, 64);
    return (threadIdx.x & 63) == 0 ? ident : __builtin_bit_cast(T, r);
}
// Exclusive scan over a workgroup of NT threads (NT / 64 <= 16 waves): DPP wave scans; the wave totals meet in
// s_w (NT / 64 entries), every wave scans them in its first row and takes its own prefix.  Barriers inside.
template <int NT, typename T, typename Op>
__device__ __forceinline__ T block_excl_scan_dpp(const T& v, const T& ident, Op op, T* s_w, T* total = nullptr) {
    constexpr int NW = NT / kWave;
    static_assert(NW >= 1 && NW <= 16, "waves");
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const T inc = wave_incl_scan(v, ident, op);
    if (lane == 63) s_w[wid] = inc;
    __syncthreads();
    T w = lane < NW ? s_w[lane] : ident;
    w = op(dpp_pod<0x111, 0xf>(w, ident), w);
    w = op(dpp_pod<0x112, 0xf>(w, ident), w);
    w = op(dpp_pod<0x114, 0xf>(w, ident), w);
    w = op(dpp_pod<0x118, 0xf>(w, ident), w);
    if (total) *total = readlane_pod(w, NW - 1);
    const T wex = wid ? readlane_pod(w, wid - 1) : ident;
    __syncthreads();                                // s_w free again
    return op(wex, shfl_up1_pod(inc, ident));
}

struct SegAgg {                                    // segmented-scan element: a thread's terms as one map
    long long d0, d1;
    int pf;                                        // p | (a segment starts inside) << 2
    int nh;                                        // heads inside
};
__device__ __forceinline__ SegAgg seg_ident() { return SegAgg{0, 0, 2, 0}; }
__device__ __forceinline__ SegAgg seg_op(const SegAgg& a, const SegAgg& b) {
    if (b.pf & 4) return SegAgg{b.d0, b.d1, b.pf, a.nh + b.nh};
    const SeqTx t = tx_then(SeqTx{a.d0, a.d1, a.pf & 3}, SeqTx{b.d0, b.d1, b.pf & 3});
    return SegAgg{t.d0, t.d1, t.p | (a.pf & 4), a.nh + b.nh};
}

constexpr int kTxHeadCap = 512;                    // heads per sum (more: the plain chain)
constexpr int kExactMergeMax = 8192;               // exact scale from presorted runs (k_rank_runs + k_exact_scale_s)
template <int NT>
struct MonoScratch {
    double wd[NT / kWave];
    SegAgg wa[NT / kWave];
    int elast[NT];                                 // predicted binade of each thread's last term
    int hedge[NT];                                 // bit 0: the thread's first term heads, bit 1: its last term heads
    int h_idx[kTxHeadCap];
    int h_e[kTxHeadCap];
    long long h_d0[kTxHeadCap];                    // the head's segment as a two-state map
    long long h_d1[kTxHeadCap];
    double result;
    int nheads, fb_seg, fb_terms;
};

// The plain chain (mono_sum_tx's fallback beyond kTxHeadCap heads): wave 0 adds s_x[0, cnt) to +0 in order.
template <int NT>
__device__ inline double chain_sum_tx(const double* s_x, int cnt, MonoScratch<NT>& S) {
    if ((threadIdx.x >> 6) == 0) {
        double s = 0.0;
        for (int j = 0; j < cnt; ++j) s = s + s_x[j];
        if (threadIdx.x == 0) S.result = s;
    }
    __syncthreads();
    return S.result;
}

// Does the prefix T lie within 2^-30 of either end of its binade?  (The true running sum differs from the predicted
// prefix by < n 2^-53 relative; terms this close to a power of two head their own segment.)
__device__ __forceinline__ bool near_edge(double T) {
    const uint64_t m = __builtin_bit_cast(uint64_t, T) & ((1ull << 52) - 1);
    return m < (1ull << 22) || m > (1ull << 52) - (1ull << 22);
}

// acc = fma(v of lane N of this 16-lane row, 1.0, acc): rounds exactly as acc + v; no LDS, no readlane.
template <int N>
__device__ __forceinline__ void bcast_add(double& acc, double v, double one) {
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(v), "v"(one), "i"(N));
}
// Heads N.. of a 16-head window (every 16-lane row holds the window's heads in lanes 0-15): the head's own step, the
// sum right after it recorded in lane N of each row, then the segment as s + u d_p (p = the low bit of s's mantissa:
// Q's parity while s lies in the head's binade, which the check afterwards confirms).
template <int N>
__device__ __forceinline__ void walk_row(double& s, double& rec, double hx, double q0, double q1, double one, int left,
                                         int n16) {
    if constexpr (N < 16) {
        if (N < left) {
            bcast_add<N>(s, hx, one);
            rec = n16 == N ? s : rec;
            double s0 = s, s1 = s;
            bcast_add<N>(s0, q0, one);
            bcast_add<N>(s1, q1, one);
            s = (__double2loint(s) & 1) ? s1 : s0;
            walk_row<N + 1>(s, rec, hx, q0, q1, one, left, n16);
        }
    }
}

// +0 + x_0 + x_1 + ... + x_{cnt-1} in index order, one fp64 rounding per addition, for x_j >= +0 (no NaN).
// One workgroup of NT threads; thread t holds terms t*PT .. t*PT + PT - 1 in x (zero past cnt) and the same terms sit in
// s_x (LDS: the walk's head terms, term-by-term fallbacks).  Heads: the first non-zero term, every non-zero term whose
// predicted binade differs from its predecessor's, lies within 2^-30 of a binade end, or is too large for the integer
// model; every other term is a step of its head's segment map.  The walk (wave 0) does a head's step directly, then its
// segment as s + u d_p when s lies in the predicted binade and the result stays below 2^(E+1); else the segment term by
// term.  False when the heads exceed kTxHeadCap (the caller sums the chain).  stamps (nullable, diagnostic builds):
// thread 0 stores s_memtime after the head count, the segmented scan and the records.
template <int NT, int PT>
__device__ __forceinline__ bool mono_sum_tx(const double (&x)[PT], int cnt, const double* s_x, MonoScratch<NT>& S,
                                            double& out, unsigned long long* stamps = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, base = tid * PT;
    // 1. approximate prefix (fp64, tree order): the prediction of each step's binade
    double run = 0.0;
#pragma unroll
    for (int a = 0; a < PT; ++a) run += x[a];
    const double tex = block_excl_scan_dpp<NT>(run, 0.0, [](double a, double b) { return a + b; }, S.wd);
    S.elast[tid] = binade64(tex + run);
    __syncthreads();
    // 2. predicted binades and heads (a term's predecessor's binade as its owner computed it)
    int E[PT];
    bool hd[PT];
    int nh = 0;
    {
        double tl = 0.0;
        int ep = tid ? S.elast[tid - 1] : kExpNone;
#pragma unroll
        for (int a = 0; a < PT; ++a) {
            tl += x[a];
            const double T = tex + tl;
            E[a] = binade64(T);
            const bool act = base + a < cnt && x[a] != 0.0;
            bool h = act && (E[a] == kExpNone || E[a] != ep || near_edge(T));
            if (act && !h) h = !(ldexp(x[a], 52 - E[a]) < 0x1p53);
            hd[a] = h;
            nh += h ? 1 : 0;
            ep = E[a];
        }
    }
    S.hedge[tid] = (hd[0] ? 1 : 0) | (hd[PT - 1] ? 2 : 0);
    __syncthreads();
    const bool prev_head = tid ? (S.hedge[tid - 1] & 2) != 0 : false;
    const bool next_head = tid + 1 < NT ? (S.hedge[tid + 1] & 1) != 0 : false;
    if (stamps && tid == 0) stamps[0] = __builtin_amdgcn_s_memtime();
    // 3. the thread's terms as one segmented map (a head's own step is the walk's: identity here), with its head count
    SegAgg agg{0, 0, 2, nh};
#pragma unroll
    for (int a = 0; a < PT; ++a) {
        if (hd[a] || (a ? hd[a - 1] : prev_head)) { agg.d0 = 0; agg.d1 = 0; agg.pf = 2 | 4; }   // a segment starts
        if (base + a < cnt && x[a] != 0.0 && !hd[a]) {
            SeqTx m{agg.d0, agg.d1, agg.pf & 3};
            tx_push(m, x[a], E[a]);
            agg.d0 = m.d0; agg.d1 = m.d1; agg.pf = m.p | (agg.pf & 4);
        }
    }
    SegAgg tot;
    const SegAgg ex = block_excl_scan_dpp<NT>(agg, seg_ident(), seg_op, S.wa, &tot);
    const int htot = tot.nh;
    if (stamps && tid == 0) stamps[1] = __builtin_amdgcn_s_memtime();
    if (htot > kTxHeadCap) return false;                       // uniform
    // 4. head records and each segment's map (written by the thread holding the segment's last term)
    {
        SeqTx cur{ex.d0, ex.d1, ex.pf & 3};
        int hk = ex.nh;
#pragma unroll
        for (int a = 0; a < PT; ++a) {
            const int j = base + a;
            if (hd[a] || (a ? hd[a - 1] : prev_head)) cur = tx_ident();
            if (j < cnt && x[a] != 0.0 && !hd[a]) tx_push(cur, x[a], E[a]);
            if (hd[a]) { S.h_idx[hk] = j; S.h_e[hk] = E[a]; ++hk; }
            const bool last = j == cnt - 1 || (j < cnt && (a + 1 < PT ? hd[a + 1] : next_head));
            if (last && hk > 0) { S.h_d0[hk - 1] = cur.d0; S.h_d1[hk - 1] = cur.d1; }
        }
    }
    __syncthreads();
    if (stamps && tid == 0) stamps[2] = __builtin_amdgcn_s_memtime();
    // 5. the walk (wave 0, wave-uniform): windows of 16 heads, every 16-lane row holding the window; a head costs a
    //    dependent fma, a parity select and a second fma (row_newbcast operands); the checks run lane-parallel after the
    //    window, and from a failed check on it goes head by head (the failed head's segment term by term)
    if (wid == 0) {
        const double one = 1.0;
        const int n16 = lane & 15;
        double s = 0.0;
        int fbs = 0, fbt = 0;
        for (int k0 = 0; k0 < htot; k0 += 16) {
            const int kk = k0 + n16;
            int hi = 0, hend = 0, E0 = kExpNone;
            long long d0 = 0, d1 = 0;
            double hx = -0.0, q0 = -0.0, q1 = -0.0;              // past the window: a no-op head (x + -0 == x)
            bool seg = false, bad = false;
            if (kk < htot) {
                hi = S.h_idx[kk];
                hend = kk + 1 < htot ? S.h_idx[kk + 1] : cnt;
                E0 = S.h_e[kk];
                hx = s_x[hi];
                seg = hend > hi + 1;
                if (seg) {
                    d0 = S.h_d0[kk];
                    d1 = S.h_d1[kk];
                    bad = E0 == kExpNone || d0 >= (1ll << 53) || d1 >= (1ll << 53);
                    if (!bad) {
                        const double u = ldexp(1.0, E0 - 52);
                        q0 = static_cast<double>(d0) * u;
                        q1 = static_cast<double>(d1) * u;
                    }
                }
            }
            // the check on the sum right after head kk's own step: s in [2^E, 2^(E+1)) and Q + d_parity <= 2^53 - 1
            auto check = [&](double sv) -> bool {
                if (!seg) return true;
                if (bad || binade64(sv) != E0) return false;
                const long long Q = static_cast<long long>((__builtin_bit_cast(uint64_t, sv) & ((1ull << 52) - 1)) | (1ull << 52));
                return Q + ((Q & 1) ? d1 : d0) <= (1ll << 53) - 1;
            };
            const int left = min(16, htot - k0);
            double rec = 0.0;
            walk_row<0>(s, rec, hx, q0, q1, one, left, n16);
            const unsigned long long badm = __ballot(!check(rec)) & 0xFFFFull;
            if (badm) {                                          // uniform
                const int f = __builtin_ctzll(badm);
                s = rl64d(rec, f);
                for (int l = f; l < left; ++l) {
                    if (l > f) s = s + rl64d(hx, l);
                    const bool ok = l > f && ((__ballot(check(s)) >> l) & 1ull) != 0ull;   // head l's own check
                    if (ok) {
                        s = s + ((__double2loint(s) & 1) ? rl64d(q1, l) : rl64d(q0, l));
                    } else {
                        const int h = __builtin_amdgcn_readlane(hi, l), end = __builtin_amdgcn_readlane(hend, l);
                        for (int j = h + 1; j < end; ++j) s = s + s_x[j];
                        fbs += end > h + 1 ? 1 : 0;
                        fbt += end - h - 1;
                    }
                }
            }
        }
        if (lane == 0) { S.result = s; S.fb_seg = fbs; S.fb_terms = fbt; S.nheads = htot; }
    }
    __syncthreads();
    out = S.result;
    return true;
}

// Sorting support for the exact scale (k_rank_runs): the number of keys of a sorted 256-key run below x (STRICT) or
// not above x -- nine probes, no branch.
template <bool STRICT>
__device__ __forceinline__ int run_count(const uint64_t* R, uint64_t x) {
    int p = 0;
#pragma unroll
    for (int s = 128; s >= 1; s >>= 1) {
        const uint64_t v = R[p + s - 1];
        p += (STRICT ? v < x : v <= x) ? s : 0;
    }
    const uint64_t v = R[p];
    return p + ((STRICT ? v < x : v <= x) ? 1 : 0);
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
// walk reaches the head) + (end - h) u / 2 (one half-ulp per step) + the fp64 error of T: when that total stays below
// M - u, every partial sum of the segment is inside the binade, one ulp from its edges, and the integer model is exact
// for each step.  Implemented across the chip for long columns below (k_mw_* in lo_exact.hip).
// ---------------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ int binade_abs(double v) {       // binade of |v| when it is a normal fp32 magnitude
    const double a = fabs(v);
    const uint64_t b = __builtin_bit_cast(uint64_t, a);
    const int f = static_cast<int>((b >> 52) & 0x7FF);
    const int e = f - 1023;
    return (a > 0.0 && f != 0x7FF && e >= -120 && e <= 126) ? e : kExpNone;
}

}  // namespace lo

namespace lo {

// ---------------------------------------------------------------------------------------------------------------------
// Long signed fp32 columns across the chip (the exact mode's 43 normal-equation sums of scans beyond kExactMaxPoints,
// up to 4M terms each).  The exact running sum is unknown until the walk reaches a term, so the phases run as
// launches over every 4096-term chunk of every column at once:
//   1. k_mw_chunk_sums: each chunk's fp64 sum and sum of magnitudes;
//   2. k_mw_drift:      each chunk's modelled rounding error: the fp32 running sum drifts from the exact prefix by the
//      sum of its step roundings, rint(x / u) u - x with u from the predicted binade -- over a long column of shrinking
//      sums the drift outgrows the checks' margin, so the prediction carries it;
//   3. k_mw_classify:   each chunk's prediction base T0 = the fp64 sum of the chunks before it plus their modelled drift,
//      its heads and integer prefix, and for every head the record the walk needs (its term, the segment's sum u * Q,
//      the check's interval) -- in HBM; k_mw_compact then lays the records out in walk order;
//   4. k_mw_walk:       one wave per column walks every head in order, 64 at a time as a plain fp32 chain (operands
//      broadcast from LDS, the next window's records in flight), then checks the 64 heads lane-parallel; from a failed
//      check on, head by head, a failed segment term by term.
// The prediction error bound eps_t is 2^-45 times (the column's sum of magnitudes up to the chunk's end + |T0|): only
// the differences T_j - T_h within a chunk enter the proof, and the chunk's own fp64 prefix is a summation tree of depth
// < 64 over its terms and T0.  Any T0 is correct -- the walk's check measures the real deviation at every head -- a good
// one keeps the segments parallel.
// ---------------------------------------------------------------------------------------------------------------------
constexpr int kMwThreads = 256;                    // classification workgroup
constexpr int kMwPT = 16;                          // consecutive terms per thread
constexpr int kMwChunk = kMwThreads * kMwPT;       // terms per chunk
constexpr int kMwCap = 1024;                       // head records per chunk (more: the chunk is one term-by-term run)
constexpr int kMwMaxChunks = 1024;                 // chunks per column the walk's LDS offset table holds
static_assert(static_cast<long long>(kMaxBlocks) * kBlock <= static_cast<long long>(kMwMaxChunks) * kMwChunk,
              "a scan of the largest size must fit the walk's offset table");
constexpr int kMwFail = 2;                         // record flag: the segment always goes term by term
constexpr int kMwPad = 128;                        // no-op records after a column's last head (the walk's loads
                                                   // run two windows ahead unconditionally)

// Head records, structure of arrays, [column][chunk][kMwCap] as classified, then [column][k] compacted in walk order;
// per-chunk sums and counts [column][chunk].  The walk's check of a multi-term segment is an interval test on the
// running sum d right after the head's step: d in [dlo, dhi] <=> the sign, the binade [2^E, 2^(E+1)) and
// |d - T| <= dev of the proof above all hold (bounds rounded inwards).
struct MwBuf {
    int* idx;          // the head's term index in the column
    int* end;          // one past its segment's last term
    float* x;          // the head's own term
    float* dq;         // the rest of the segment, u * Q (exact in fp32 whenever the check passes; -0 for one term)
    int* flag;         // 1: passes any check (one-term segment), kMwFail: never passes; else 0
    double* dlo;       // the check's interval
    double* dhi;
    int* c_idx;        // the same records compacted: [column][k], k over every head of the column in order
    int* c_end;
    float* c_x;
    float* c_dq;
    int* c_flag;
    double* c_dlo;
    double* c_dhi;
    int* nh;           // heads per chunk
    int* ntot;         // heads per column (k_mw_compact)
    double* csum;      // chunk sums (fp64)
    double* cabs;      // chunk sums of magnitudes
    double* dcorr;     // chunk sums of the modelled fp32 rounding errors (the prediction's drift correction)
    int nchunks;       // chunks per column (the row stride of nh / csum / cabs; records: nchunks * kMwCap)
    size_t cstride;    // column stride of the compacted records: nchunks * kMwCap + kMwPad
};

}  // namespace lo

namespace lo {

// Long non-negative fp64 sums across the chip (the iteration-0 scale of scans beyond kExactMaxPoints: the sorted
// residuals' sum, then the sum of (r - mean)^2 -- IterativeClosestPointOptimizer.cpp:304-316).  mono_seq_sum's method
// spread like the signed columns above: chunk sums -> classification (heads at predicted binade changes and halfway
// ties, integer prefix sums) -> compaction -> one wave walking the heads.  A mono segment's check is exact and needs no
// prediction bound: the sum right after the head's step lies in [2^E, 2^(E+1) - u - u * Q].
constexpr int kMwmCap = kMwChunk;                  // mono: every term may head (halfway ties are common: residuals
                                                   // carry ~40 significant bits), so no chunk runs term by term
struct MwmBuf {
    int* idx;          // records as classified, [chunk][kMwCap]
    int* end;
    int* flag;         // 1: passes any check, kMwFail: never passes, else 0
    double* x;         // the head's own term
    double* dq;        // u * Q (-0 for a one-term segment)
    double* dlo;       // the check's interval on the sum right after the head's step
    double* dhi;
    int* c_idx;        // compacted in walk order
    int* c_end;
    int* c_flag;
    double* c_x;
    double* c_dq;
    double* c_dlo;
    double* c_dhi;
    int* nh;           // heads per chunk
    double* csum;      // chunk sums (fp64)
    int* cnt;          // [0]: accepted residuals (the finite prefix of the sorted array); [1]: any NaN; [2]: heads in total
    double* res;       // [0]: the sum; [1]: the variance sum
    int nchunks;
};

}  // namespace lo
