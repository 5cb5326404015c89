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
// Halfway ties without heads (mono_sum_tx below).
// Inside binade E the running sum is s = Q u (u = 2^(E-52), Q in [2^52, 2^53)), and a term x = m 2^(e-52) (m its 53-bit
// integer mantissa) adds t = x / u = m 2^(e-E): Q gains f = m >> (E-e), plus one when the dropped bits are above half --
// unless they are exactly half (a tie), where round-half-even gives Q + f when Q + f is even and Q + f + 1 otherwise,
// and leaves Q even.  So inside a segment (the steps after a head, all in the head's predicted binade) only the FIRST
// tie depends on the parity Q had when the segment started: every later tie sees Q even after the previous tie, plus
// the parities of the plain steps since.  A term's increment is thus known from its own bits and the XOR of the
// increment parities back to the last tie or head (a segmented XOR scan of single bits), except the first tie's +1,
// which the walk decides from the entry parity (the segment record keeps c1 = that XOR ^ the tie's f parity).  Segment
// totals are differences of one int64 prefix sum; everything per term is integer arithmetic on the mantissa bits.
// ---------------------------------------------------------------------------------------------------------------------
struct TermBits {
    long long f;             // floor(x / u); 2^62 when x / u >= 2^53 (never a segment step: the head rule)
    int tie, up;             // the dropped bits are exactly half / above half
};
__device__ __forceinline__ TermBits term_bits(double x, int E) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    const int ef = static_cast<int>((b >> 52) & 0x7FF);
    const uint64_t m = (b & ((1ull << 52) - 1)) | (ef ? (1ull << 52) : 0ull);
    const int k = E - (ef ? ef - 1023 : -1022);             // x = m 2^(e-52): t = m 2^-k
    TermBits r{0, 0, 0};
    if (k <= 0) {
        r.f = k == 0 ? static_cast<long long>(m) : (1ll << 62);
    } else if (k < 54) {
        r.f = static_cast<long long>(m >> k);
        const uint64_t rem = m & ((1ull << k) - 1), half = 1ull << (k - 1);
        r.tie = rem == half ? 1 : 0;
        r.up = rem > half ? 1 : 0;
    }                                                         // k >= 54: t < 1/2 (m < 2^53 <= the half bit)
    return r;
}
// The segmented XOR-scan state, four bits: 1 a reset (tie or head) inside, 2 the XOR of plain-step parities since the
// last reset (or since the start), 4 a head inside, 8 a tie since the last head (or since the start).
__device__ __forceinline__ int xs_op(int a, int b) {       // a, then b
    const int x = (b & 1) ? (b & 2) : ((a ^ b) & 2);
    const int t = (b & 4) ? (b & 8) : ((a | b) & 8);
    return ((a | b) & 5) | x | t;
}

// Wave-wide inclusive scan of a POD of 32-bit words by DPP (row_shr 1/2/4/8, then row_bcast 15/31 into the upper
// rows): the earlier lane's value is combined in front, op(earlier, later).  Lanes without a source keep `ident`.
template <int N> struct Words { int w[N]; };
template <int CTRL, int RM, typename T>
__device__ __forceinline__ T dpp_pod(T v, T old) {
    static_assert(sizeof(T) % 4 == 0, "32-bit words");
    constexpr int N = sizeof(T) / 4;
    const Words<N> a = __builtin_bit_cast(Words<N>, v), o = __builtin_bit_cast(Words<N>, old);
    Words<N> r;
#pragma unroll
    for (int i = 0; i < N; ++i) r.w[i] = __builtin_amdgcn_update_dpp(o.w[i], a.w[i], CTRL, RM, 0xf, false);
    return __builtin_bit_cast(T, r);
}
template <typename T, typename Op>
__device__ __forceinline__ T wave_incl_scan(T v, T ident, Op op) {
    v = op(dpp_pod<0x111, 0xf>(v, ident), v);       // row_shr:1
    v = op(dpp_pod<0x112, 0xf>(v, ident), v);       // row_shr:2
    v = op(dpp_pod<0x114, 0xf>(v, ident), v);       // row_shr:4
    v = op(dpp_pod<0x118, 0xf>(v, ident), v);       // row_shr:8   (16-lane rows scanned)
    v = op(dpp_pod<0x142, 0xa>(v, ident), v);       // row_bcast:15 into rows 1, 3
    v = op(dpp_pod<0x143, 0xc>(v, ident), v);       // row_bcast:31 into rows 2, 3
    return v;
}
template <typename T>
__device__ __forceinline__ T readlane_pod(T v, int l) {
    constexpr int N = sizeof(T) / 4;
    Words<N> a = __builtin_bit_cast(Words<N>, v);
#pragma unroll
    for (int i = 0; i < N; ++i) a.w[i] = __builtin_amdgcn_readlane(a.w[i], l);
    return __builtin_bit_cast(T, a);
}
template <typename T>
__device__ __forceinline__ T shfl_up1_pod(T v, T ident) {
    constexpr int N = sizeof(T) / 4;
    const Words<N> a = __builtin_bit_cast(Words<N>, v), o = __builtin_bit_cast(Words<N>, ident);
    const bool first = (threadIdx.x & 63) == 0;
    Words<N> r;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const int t = __shfl_up(a.w[i], 1, 64);
        r.w[i] = first ? o.w[i] : t;
    }
    return __builtin_bit_cast(T, r);
}
// Exclusive scan over a workgroup of NT threads (NT / 64 <= 16 waves): DPP wave scans; the wave totals meet in
// s_w (NT / 64 entries), every wave scans them in its first row and takes its own prefix.  Two barriers.
template <int NT, typename T, typename Op>
__device__ __forceinline__ T block_excl_scan_dpp(T v, T ident, Op op, T* s_w, T* total = nullptr) {
    constexpr int NW = NT / kWave;
    static_assert(NW >= 1 && NW <= 16, "waves");
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const T inc = wave_incl_scan(v, ident, op);
    const T ex = shfl_up1_pod(inc, ident);
    if constexpr (NW == 1) {
        if (total) *total = readlane_pod(inc, 63);
        return ex;
    }
    if (lane == 63) s_w[wid] = inc;
    __syncthreads();
    T w = lane < NW ? s_w[lane] : ident;
#pragma unroll
    for (int sh = 1; sh < NW; sh <<= 1) {
        if (sh == 1) w = op(dpp_pod<0x111, 0xf>(w, ident), w);
        if (sh == 2) w = op(dpp_pod<0x112, 0xf>(w, ident), w);
        if (sh == 4) w = op(dpp_pod<0x114, 0xf>(w, ident), w);
        if (sh == 8) w = op(dpp_pod<0x118, 0xf>(w, ident), w);
    }
    if (total) *total = readlane_pod(w, NW - 1);
    const T wex = wid ? readlane_pod(w, wid - 1) : ident;
    __syncthreads();                                // s_w free again
    return wid ? op(wex, ex) : ex;
}

constexpr int kTxHeadCap = 256;                    // heads per sum (more: the plain chain)
constexpr int kTxAny = 100000;                     // walk record: a head without a segment (every check passes)
constexpr int kExactMergeMax = 8192;               // exact scale from presorted runs (k_rank_runs + k_exact_scale_s)
template <int NT>
struct MonoScratch {
    double wd[NT / kWave];
    long long wl[NT / kWave];
    int wi[NT / kWave];
    int welast[NT / kWave];                        // predicted binade of each wave's last term
    int h_idx[kTxHeadCap];
    int h_e[kTxHeadCap];
    long long h_p[kTxHeadCap];                     // the int64 prefix of the increments at the head
    int h_c1[kTxHeadCap];                          // bit 1: the segment has a tie, bit 0: c1 of its first tie
    double w_hx[kTxHeadCap];                       // the walk's records: the head's term, u d_0, u d_1,
    double w_q0[kTxHeadCap];
    double w_q1[kTxHeadCap];
    long long w_d0[kTxHeadCap];                    //   d_0, d_1, the check's binade (kTxAny: no segment), the segment's end
    long long w_d1[kTxHeadCap];
    int w_e[kTxHeadCap];
    int w_end[kTxHeadCap];
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
// predicted binade differs from its predecessor's, lies within 2^-30 of a binade end, or steps by 2^49 units or more;
// every other term is an integer step of its head's segment.  Three block scans (the fp64 prediction, the 4-bit XOR
// state, the int64 increments), then the walk (wave 0): a head's step done directly, its segment as s + u d_p (p = Q's
// parity at the segment's start, d_p = the segment's increments with the first tie's +1 for that parity) when s lies in
// the predicted binade and the result stays below 2^(E+1); else the segment term by term.  False when the heads exceed
// kTxHeadCap (the caller sums the chain).  stamps (nullable, diagnostic builds): thread 0 stores s_memtime after the
// heads, the scans and the records.
template <int NT, int PT>
__device__ __forceinline__ bool mono_sum_tx(const double (&x)[PT], int cnt, const double* s_x, MonoScratch<NT>& S,
                                            double& out, unsigned long long* stamps = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, base = tid * PT;
    // 1. approximate prefix (fp64): the prediction of each step's binade
    double run = 0.0;
#pragma unroll
    for (int a = 0; a < PT; ++a) run += x[a];
    const double tex = block_excl_scan_dpp<NT>(run, 0.0, [](double a, double b) { return a + b; }, S.wd);
    // 2. predicted binades, integer steps and heads; a term's predecessor's binade as its owner computed it (lane
    //    l - 1's last term; lane 0: the previous wave's, through LDS)
    int E[PT];
    TermBits tb[PT];
    bool hd[PT];
    int nh = 0;
    double tl = 0.0;
#pragma unroll
    for (int a = 0; a < PT; ++a) {
        tl += x[a];
        E[a] = binade64(tex + tl);
    }
    const int e_up = __shfl_up(E[PT - 1], 1, 64);
    if (lane == 63) S.welast[wid] = E[PT - 1];
    __syncthreads();
    {
        int ep = lane ? e_up : (wid ? S.welast[wid - 1] : kExpNone);
        tl = 0.0;
#pragma unroll
        for (int a = 0; a < PT; ++a) {
            tl += x[a];
            const bool act = base + a < cnt && x[a] != 0.0;
            tb[a] = term_bits(x[a], E[a] == kExpNone ? 0 : E[a]);
            const bool h = act && (E[a] == kExpNone || E[a] != ep || near_edge(tex + tl) || tb[a].f >= (1ll << 49));
            hd[a] = h;
            nh += h ? 1 : 0;
            ep = E[a];
        }
    }
    // 3. the segmented XOR state over the thread's terms (bits 0-3, xs_op) with the thread's head count above them
    auto bits_of = [&](int a) -> int {                      // a term's own 4-bit state
        if (hd[a]) return 1 | 4;
        if (!(base + a < cnt && x[a] != 0.0)) return 0;
        if (tb[a].tie) return 1 | 8;
        return static_cast<int>((tb[a].f + tb[a].up) & 1) << 1;
    };
    int xs = 0;
#pragma unroll
    for (int a = 0; a < PT; ++a) xs = xs_op(xs, bits_of(a));
    int xtot = 0;
    const int xex = block_excl_scan_dpp<NT>(xs | (nh << 4), 0,
                                            [](int a, int b) { return xs_op(a & 15, b & 15) | (((a >> 4) + (b >> 4)) << 4); },
                                            S.wi, &xtot);
    const int hbase = xex >> 4, htot = xtot >> 4;
    if (stamps && tid == 0) stamps[0] = __builtin_amdgcn_s_memtime();
    // 4. each term's increment (a tie after another tie of its segment: f + (XOR ^ f's parity); the first tie: f, the
    //    +1 left to the walk), the thread's total, the int64 prefix
    long long inc_tot = 0;
    {
        int st = xex & 15;
#pragma unroll
        for (int a = 0; a < PT; ++a) {
            const bool act = base + a < cnt && x[a] != 0.0 && !hd[a];
            long long inc = 0;
            if (act) {
                if (tb[a].tie) inc = tb[a].f + ((st & 8) ? (((st >> 1) ^ static_cast<int>(tb[a].f)) & 1) : 0);
                else inc = tb[a].f + tb[a].up;
            }
            inc_tot += inc;
            st = xs_op(st, bits_of(a));
        }
    }
    if (htot > kTxHeadCap) return false;                       // uniform
    for (int k = tid; k < htot; k += NT) S.h_c1[k] = 0;       // ordered before step 5 by the scan's barriers
    long long ptot = 0;
    const long long pex = block_excl_scan_dpp<NT>(inc_tot, 0ll, [](long long a, long long b) { return a + b; }, S.wl, &ptot);
    if (stamps && tid == 0) stamps[1] = __builtin_amdgcn_s_memtime();
    // 5. head records (index, binade, the prefix at the head) and each segment's first tie (c1)
    {
        int st = xex & 15;
        long long P = pex;
        int hk = hbase;
#pragma unroll
        for (int a = 0; a < PT; ++a) {
            const int j = base + a;
            const bool act = j < cnt && x[a] != 0.0 && !hd[a];
            if (hd[a]) { S.h_idx[hk] = j; S.h_e[hk] = E[a]; S.h_p[hk] = P; ++hk; }
            long long inc = 0;
            if (act) {
                if (tb[a].tie) {
                    if (st & 8) inc = tb[a].f + (((st >> 1) ^ static_cast<int>(tb[a].f)) & 1);
                    else {
                        inc = tb[a].f;
                        if (hk > 0) S.h_c1[hk - 1] = 2 | (((st >> 1) ^ static_cast<int>(tb[a].f)) & 1);
                    }
                } else {
                    inc = tb[a].f + tb[a].up;
                }
            }
            P += inc;
            st = xs_op(st, bits_of(a));
        }
    }
    __syncthreads();
    // 6. every head's walk record, in parallel: its term, its segment's increments for either entry parity as fp64
    //    multiples of u (exact below 2^53), the check's binade and increments (E = kExpNone: never passes; a head
    //    without a segment: always passes)
    for (int k = tid; k < htot; k += NT) {
        const int hi = S.h_idx[k], hend = k + 1 < htot ? S.h_idx[k + 1] : cnt, E0 = S.h_e[k];
        double q0 = -0.0, q1 = -0.0;                           // x + -0 == x for every x
        int e = kTxAny;
        long long d0 = 0, d1 = 0;
        if (hend > hi + 1) {
            const long long D = (k + 1 < htot ? S.h_p[k + 1] : ptot) - S.h_p[k];
            const int c = S.h_c1[k];
            d0 = D + ((c & 2) ? (c & 1) : 0);
            d1 = D + ((c & 2) ? ((c & 1) ^ 1) : 0);
            e = (E0 == kExpNone || D < 0 || d0 >= (1ll << 53) || d1 >= (1ll << 53)) ? kExpNone : E0;
            if (e != kExpNone) {
                const double u = ldexp(1.0, E0 - 52);
                q0 = static_cast<double>(d0) * u;
                q1 = static_cast<double>(d1) * u;
            }
        }
        S.w_hx[k] = s_x[hi];
        S.w_q0[k] = q0;
        S.w_q1[k] = q1;
        S.w_e[k] = e;
        S.w_end[k] = hend;
        S.w_d0[k] = d0;
        S.w_d1[k] = d1;
    }
    __syncthreads();
    if (stamps && tid == 0) stamps[2] = __builtin_amdgcn_s_memtime();
    // 7. the walk (wave 0, wave-uniform): windows of 16 heads, every 16-lane row holding the window; a head costs a
    //    dependent fma, a parity select and a second fma (row_newbcast operands); the checks run lane-parallel after the
    //    window, and from a failed check on it goes head by head (the failed head's segment term by term)
    if (wid == 0) {
        const double one = 1.0;
        const int n16 = lane & 15;
        double s = 0.0;
        int fbs = 0, fbt = 0;
        for (int k0 = 0; k0 < htot; k0 += 16) {
            const int kk = k0 + n16;
            const bool in = kk < htot;
            const double hx = in ? S.w_hx[kk] : -0.0, q0 = in ? S.w_q0[kk] : -0.0, q1 = in ? S.w_q1[kk] : -0.0;
            const int e = in ? S.w_e[kk] : kTxAny;
            const long long d0 = in ? S.w_d0[kk] : 0, d1 = in ? S.w_d1[kk] : 0;
            // the check on the sum right after head kk's own step: s in [2^E, 2^(E+1)) and Q + d_parity <= 2^53 - 1
            auto check = [&](double sv) -> bool {
                if (e == kTxAny) return true;
                if (binade64(sv) != e) return false;               // also kExpNone (never a valid binade)
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
                        const int h = S.h_idx[k0 + l], end = S.w_end[k0 + l];
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
// not above x, for every run at once (the runs' nine-probe binary searches interleaved: NR loads in flight per probe).
template <int NR>
__device__ __forceinline__ int runs_rank(const uint64_t* s_r, int nb, int b, uint64_t x) {
    int p[NR];
    bool use[NR], le[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        p[r] = (r < nb ? r : 0) * 256;                     // a row past nb reads row 0 and is not counted
        use[r] = r < nb && r != b;
        le[r] = r < b;                                     // earlier runs: keys not above x; later runs: below x
    }
#pragma unroll
    for (int st = 128; st >= 1; st >>= 1) {
        uint64_t v[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) v[r] = s_r[p[r] + st - 1];
#pragma unroll
        for (int r = 0; r < NR; ++r) p[r] += (le[r] ? v[r] <= x : v[r] < x) ? st : 0;
    }
    int rank = 0;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const uint64_t v = s_r[p[r]];
        const int c = (p[r] & 255) + ((le[r] ? v <= x : v < x) ? 1 : 0);
        rank += use[r] ? c : 0;
    }
    return rank;
}


}  // namespace lo

namespace lo {

// ---------------------------------------------------------------------------------------------------------------------
// Signed fp32 sequential sums (the reference's build_ne accumulates H, g and the cost as running fp32 sums,
// IterativeClosestPointOptimizer.cpp:359-415).  The same idea as mono_seq_sum, for terms of either sign: while the
// running sum s keeps its sign and binade [2^E, 2^(E+1)) in magnitude, fl(s + x) = s + u rint(x / u), u = 2^(E-23).
// The partial sums of a segment are no longer monotone, so the prediction carries the proof: a term heads a segment
// also when its predicted prefix T lies within M = 2^(E-10) of either edge of its binade (kMwEdgeBits, lo_exact.hip).  Inside a segment every T_j
// is then at least M from the edges, and the true partial sums differ from T_j by at most |s_h - T_h| (known once the
// walk reaches the head) + (end - h) u / 2 (one half-ulp per step) + the fp64 error of T: when that total stays below
// M - u, every partial sum of the segment is inside the binade, one ulp from its edges, and the integer model is exact
// for each step.  Implemented across the chip for long columns below (k_mw_* in lo_exact.hip).
// ---------------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ int binade_abs(double v) {       // binade of |v| when it is a normal fp32 magnitude
    const uint32_t f = static_cast<uint32_t>(__builtin_bit_cast(uint64_t, v) >> 52) & 0x7FFu;   // biased exponent
    return f - 903u <= 246u ? static_cast<int>(f) - 1023 : kExpNone;   // e in [-120, 126]: zero, subnormal, inf, NaN out
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
// spread like the signed columns above: chunk sums -> classification (heads at predicted binade changes, integer
// prefix sums; halfway ties inside a segment as mono_sum_tx's two-state segments: the record carries the segment's
// increments for either parity of Q at its start) -> compaction -> one wave walking the heads.  A mono segment's check
// is exact and needs no prediction bound: the sum right after the head's step lies in [2^E, 2^(E+1) - u - u * d_p],
// p = that sum's mantissa parity.
constexpr int kMwmCap = kMwChunk;                  // mono: every term may head, so no chunk runs term by term
struct MwmBuf {
    int* idx;          // records as classified, [chunk][kMwCap]
    int* end;
    int* flag;         // 1: passes any check, kMwFail: never passes, else 0
    double* x;         // the head's own term
    double* dq;        // u * d_0: the segment's increments when Q is even at its start (-0 for a one-term segment)
    double* dq1;       // u * d_1: ... when Q is odd
    double* dlo;       // the check's interval on the sum right after the head's step: [dlo, dhi_p]
    double* dhi;
    double* dhi1;
    int* c_idx;        // compacted in walk order
    int* c_end;
    int* c_flag;
    double* c_x;
    double* c_dq;
    double* c_dq1;
    double* c_dlo;
    double* c_dhi;
    double* c_dhi1;
    int* nh;           // heads per chunk
    double* csum;      // chunk sums (fp64)
    int* cnt;          // [0]: accepted residuals (the finite prefix of the sorted array); [1]: any NaN; [2]: heads in total
    double* res;       // [0]: the sum; [1]: the variance sum
    int nchunks;
};

}  // namespace lo
