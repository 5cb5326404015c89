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
// no NaN; +inf is never among the first cnt terms).  Thread t holds terms t*PT .. t*PT + PT - 1 in x[] (zeros past
// cnt) and the same terms sit in s_x[0, cnt) (LDS; read by the walk and the fallbacks).  Carry-in for chunked use:
// T0 = the approximate prefix before term 0, e0 = the predicted binade of the term before term 0, head0 = term 0 starts
// a segment whatever its binade.  Every thread returns the sum; *e_last (nullable) receives the predicted binade of
// term cnt - 1 for the next chunk.  Returns false (nothing computed) when a pass has more than kSeqHeadCap heads.
template <int PT>
__device__ bool mono_seq_sum(const double (&x)[PT], int cnt, const double* s_x, SeqScratch& S, double T0, int e0,
                             bool head0, double s_in, double& s_out, double* T_out) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int base = tid * PT;
    // 1. approximate inclusive prefix -> predicted binade per term
    double tl[PT];
    double run = 0.0;
#pragma unroll
    for (int a = 0; a < PT; ++a) {
        run += (base + a < cnt) ? x[a] : 0.0;
        tl[a] = run;
    }
    double ttot;
    const double tex = T0 + block_excl_scan<double>(run, S.wd, ttot);
    int e[PT];
#pragma unroll
    for (int a = 0; a < PT; ++a) e[a] = binade64(tex + tl[a]);
    S.elast[tid] = e[PT - 1];
    __syncthreads();
    int ep = tid ? S.elast[tid - 1] : e0;
    // 2. heads and integer steps
    long long q[PT];
    bool hd[PT];
    long long ql = 0;
    int nhl = 0;
#pragma unroll
    for (int a = 0; a < PT; ++a) {
        const int j = base + a;
        bool head = false;
        long long qa = 0;
        if (j < cnt && (x[a] != 0.0 || (head0 && j == 0))) {   // a chunk's first term heads it even when zero
            const int E = e[a];
            if (E < -1000 || E != ep || (head0 && j == 0)) {
                head = true;
            } else {
                const double t = ldexp(x[a], 52 - E);            // exact power-of-two scaling
                const double f = floor(t), fr = t - f;           // exact (t < 2^54)
                if (fr == 0.5) head = true;                      // halfway: the rounding depends on s's last bit
                else qa = static_cast<long long>(f) + (fr > 0.5 ? 1 : 0);
            }
        }
        ep = e[a];
        hd[a] = head;
        q[a] = qa;
        ql += qa;
        nhl += head ? 1 : 0;
    }
    long long ptot;
    const long long pex = block_excl_scan<long long>(ql, S.wl, ptot);
    int htot;
    const int hbase = block_excl_scan<int>(nhl, S.wi, htot);
    if (htot > kSeqHeadCap) return false;                       // uniform: every thread sees htot
    long long prun = pex;
    int hk = hbase;
#pragma unroll
    for (int a = 0; a < PT; ++a) {
        prun += q[a];
        if (hd[a]) { S.h_idx[hk] = base + a; S.h_e[hk] = e[a]; S.h_p[hk] = prun; ++hk; }
    }
    if (tid == kSeqThreads - 1) S.e_carry = e[PT - 1];
    if (tid == 0) S.nheads = htot;
    __syncthreads();
    // 3. the walk (wave 0, wave-uniform): lane l of a 64-head window holds head k0 + l
    if (wid == 0) {
        double s = s_in;
        int fbs = 0, fbt = 0;
        for (int k0 = 0; k0 < htot; k0 += 64) {
            const int kk = k0 + lane;
            int hi = 0, he = 0, hend = cnt;
            long long hp = 0, pend = ptot;
            double hx = 0.0;
            if (kk < htot) {
                hi = S.h_idx[kk];
                he = S.h_e[kk];
                hp = S.h_p[kk];
                hx = s_x[hi];
                if (kk + 1 < htot) { pend = S.h_p[kk + 1]; hend = S.h_idx[kk + 1]; }
            }
            const int m = min(64, htot - k0);
            for (int l = 0; l < m; ++l) {
                const int h = __builtin_amdgcn_readlane(hi, l), end = __builtin_amdgcn_readlane(hend, l);
                const int E = __builtin_amdgcn_readlane(he, l);
                const long long Q = rl64i(pend, l) - rl64i(hp, l);
                s = s + rl64d(hx, l);                            // the head's own step, as the reference does it
                if (end > h + 1) {
                    const double u = ldexp(1.0, E - 52);
                    const double top = ldexp(1.0, E + 1) - u;
                    const double R = s + static_cast<double>(Q) * u;
                    if (binade64(s) == E && E >= -1000 && R <= top) {
                        s = R;                                   // every step of the segment: s + u * q_j, exact
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
    if (T_out) *T_out = T0 + ttot;
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

// Ascending bitonic sort of NT * PT doubles, thread t holding elements t*PT .. t*PT + PT - 1 (blocked): partner
// distances below PT inside the thread's registers, below 64 * PT across the wave (lane_xor: DPP / permlane swaps),
// larger ones through s_x (LDS, NT * PT doubles).  No NaN in the input (+inf sorts last).
template <int PT, int J>
__device__ __forceinline__ void bitonic_reg(double (&v)[PT], int base, int k) {
    if constexpr (J < PT) {
#pragma unroll
        for (int a = 0; a < PT; ++a) {
            if ((a & J) == 0) {
                const bool asc = ((base + a) & k) == 0;
                const double lo = v[a], hi = v[a + J];
                const bool sw = asc ? (lo > hi) : (lo < hi);
                v[a] = sw ? hi : lo;
                v[a + J] = sw ? lo : hi;
            }
        }
    }
}
// v of lane (lane ^ M) without the LDS crossbar (a ds_bpermute per 32-bit word was the sort's bottleneck): DPP
// quad_perm for M = 1, 2, row_ror:8 for 8, two row rotations and a per-lane select for 4 (which rotation brings lane
// l ^ 4 is read off the lane index itself), v_permlane16_swap / v_permlane32_swap for 16 / 32.
template <int M>
__device__ __forceinline__ double lane_xor(double v, bool sel4) {
    if constexpr (M == 1) return dpp64<0xB1, 0xf>(v);
    else if constexpr (M == 2) return dpp64<0x4E, 0xf>(v);
    else if constexpr (M == 8) return dpp64<0x128, 0xf>(v);
    else if constexpr (M == 4) {
        const double a = dpp64<0x124, 0xf>(v), b = dpp64<0x12C, 0xf>(v);   // row_ror:4, row_ror:12
        return sel4 ? a : b;
    } else {
        const unsigned lo = static_cast<unsigned>(__double2loint(v)), hi = static_cast<unsigned>(__double2hiint(v));
        const bool upper = ((threadIdx.x & 63) & M) != 0;
        if constexpr (M == 16) {
            const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
            const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
            // with both operands v: [0] holds rows (0 0 2 2), [1] rows (1 1 3 3); an even row's partner is in [1]
            return upper ? __hiloint2double(static_cast<int>(h[0]), static_cast<int>(l[0]))
                         : __hiloint2double(static_cast<int>(h[1]), static_cast<int>(l[1]));
        } else {
            static_assert(M == 32, "lane distance");
            const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
            const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
            // [0] = (lanes 0-31, lanes 0-31), [1] = (lanes 32-63, lanes 32-63)
            return upper ? __hiloint2double(static_cast<int>(h[0]), static_cast<int>(l[0]))
                         : __hiloint2double(static_cast<int>(h[1]), static_cast<int>(l[1]));
        }
    }
}
template <int PT, int M>
__device__ __forceinline__ void bitonic_lane(double (&v)[PT], int base, int k, int j, bool sel4) {
#pragma unroll
    for (int a = 0; a < PT; ++a) {
        const double o = lane_xor<M>(v[a], sel4);
        const int el = base + a;
        const bool keep_min = ((el & j) == 0) == ((el & k) == 0);
        const double mn = (o < v[a]) ? o : v[a], mx = (o > v[a]) ? o : v[a];
        v[a] = keep_min ? mn : mx;
    }
}
template <int PT>
__device__ void bitonic_sort_block(double (&v)[PT], double* s_x) {
    constexpr int N = kSeqThreads * PT;
    const int tid = threadIdx.x, base = tid * PT, lane = tid & 63;
    // which of row_ror:4 / row_ror:12 brings lane ^ 4 (the rotation direction read off the lane index)
    const bool sel4 = dpp32m<0x124>(lane) == (lane ^ 4);
    for (int k = 2; k <= N; k <<= 1) {
        int j = k >> 1;
        if (j >= 64 * PT) {
            // LDS stages of this k: pairs (p with bit j clear, p | j), each thread PT / 2 pairs per stage
#pragma unroll
            for (int a = 0; a < PT; ++a) s_x[base + a] = v[a];
            __syncthreads();
            for (; j >= 64 * PT; j >>= 1) {
                for (int p = tid; p < N / 2; p += kSeqThreads) {
                    const int lo_i = ((p & ~(j - 1)) << 1) | (p & (j - 1)), hi_i = lo_i | j;
                    const bool asc = (lo_i & k) == 0;
                    const double a0 = s_x[lo_i], a1 = s_x[hi_i];
                    const bool sw = asc ? (a0 > a1) : (a0 < a1);
                    if (sw) { s_x[lo_i] = a1; s_x[hi_i] = a0; }
                }
                __syncthreads();
            }
#pragma unroll
            for (int a = 0; a < PT; ++a) v[a] = s_x[base + a];
            __syncthreads();
        }
        for (; j >= PT; j >>= 1) {
            switch (j / PT) {                                    // partner lane = lane ^ (j / PT)
                case 32: bitonic_lane<PT, 32>(v, base, k, j, sel4); break;
                case 16: bitonic_lane<PT, 16>(v, base, k, j, sel4); break;
                case 8: bitonic_lane<PT, 8>(v, base, k, j, sel4); break;
                case 4: bitonic_lane<PT, 4>(v, base, k, j, sel4); break;
                case 2: bitonic_lane<PT, 2>(v, base, k, j, sel4); break;
                default: bitonic_lane<PT, 1>(v, base, k, j, sel4); break;
            }
        }
        // j < PT: inside the thread
        if (j >= 8) bitonic_reg<PT, 8>(v, base, k);
        if (j >= 4) bitonic_reg<PT, 4>(v, base, k);
        if (j >= 2) bitonic_reg<PT, 2>(v, base, k);
        if (j >= 1) bitonic_reg<PT, 1>(v, base, k);
    }
}

}  // namespace lo

namespace lo {

// ---------------------------------------------------------------------------------------------------------------------
// Signed fp32 sequential sums (the reference's build_ne accumulates H, g and the cost as running fp32 sums,
// IterativeClosestPointOptimizer.cpp:359-415).  The same idea as mono_seq_sum, for terms of either sign: while the
// running sum s keeps its sign and binade [2^E, 2^(E+1)) in magnitude, fl(s + x) = s + u rint(x / u) with u = 2^(E-23).
// A segment's partial sums are no longer monotone, so its check bounds the smallest and the largest integer prefix over
// the segment (segment minima / maxima by LDS atomics), and a segment also ends where the predicted sign changes.
// Terms come in chunks (kSeqThreads * PT), each chunk starting a segment; the walk carries s from chunk to chunk.
// ---------------------------------------------------------------------------------------------------------------------
constexpr int kSHeadCap = 2048;

struct SeqScratchS {
    double wd[kSeqWaves];
    long long wl[kSeqWaves];
    int wi[kSeqWaves];
    int elast[kSeqThreads];
    int glast[kSeqThreads];
    int h_idx[kSHeadCap];
    int h_e[kSHeadCap];
    int h_g[kSHeadCap];
    long long h_p[kSHeadCap];
    long long h_min[kSHeadCap];
    long long h_max[kSHeadCap];
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
// cnt), s_x[0, cnt) the same terms (LDS).  T0 / e0 / g0: the approximate prefix, predicted binade and sign carried in
// from the previous chunk; term 0 always starts a segment.  Every thread returns the sum and the carries; false (nothing
// computed) when the chunk has more than kSHeadCap heads.
template <int PT>
__device__ bool signed_seq_sum(const float (&x)[PT], int cnt, const float* s_x, SeqScratchS& S, double T0, int e0,
                               int g0, float s_in, float& s_out, double& T_out, int& e_out, int& g_out) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int base = tid * PT;
    double tl[PT];
    double run = 0.0;
#pragma unroll
    for (int a = 0; a < PT; ++a) {
        run += (base + a < cnt) ? static_cast<double>(x[a]) : 0.0;
        tl[a] = run;
    }
    double ttot;
    const double tex = T0 + block_excl_scan<double>(run, S.wd, ttot);
    int e[PT], g[PT];
#pragma unroll
    for (int a = 0; a < PT; ++a) {
        const double T = tex + tl[a];
        e[a] = binade_abs(T);
        g[a] = T > 0.0 ? 1 : (T < 0.0 ? -1 : 0);
    }
    S.elast[tid] = e[PT - 1];
    S.glast[tid] = g[PT - 1];
    __syncthreads();
    int ep = tid ? S.elast[tid - 1] : e0, gp = tid ? S.glast[tid - 1] : g0;
    long long q[PT];
    bool hd[PT];
    long long ql = 0;
    int nhl = 0;
#pragma unroll
    for (int a = 0; a < PT; ++a) {
        const int j = base + a;
        bool head = false;
        long long qa = 0;
        if (j < cnt && (x[a] != 0.0f || j == 0)) {             // a chunk's first term heads it even when zero
            const int E = e[a];
            if (E == kExpNone || E != ep || g[a] != gp || j == 0) {
                head = true;
            } else {
                const double t = ldexp(static_cast<double>(x[a]), 23 - E);   // exact
                const double f = floor(t), fr = t - f;
                if (fr == 0.5) head = true;
                else qa = static_cast<long long>(f) + (fr > 0.5 ? 1 : 0);
            }
        }
        ep = e[a];
        gp = g[a];
        hd[a] = head;
        q[a] = qa;
        ql += qa;
        nhl += head ? 1 : 0;
    }
    long long ptot;
    const long long pex = block_excl_scan<long long>(ql, S.wl, ptot);
    int htot;
    const int hbase = block_excl_scan<int>(nhl, S.wi, htot);
    if (htot > kSHeadCap) return false;
    for (int k = tid; k < htot; k += kSeqThreads) { S.h_min[k] = LLONG_MAX; S.h_max[k] = LLONG_MIN; }
    long long prun = pex;
    int hk = hbase;
    long long P[PT];
#pragma unroll
    for (int a = 0; a < PT; ++a) {
        prun += q[a];
        P[a] = prun;
        if (hd[a]) { S.h_idx[hk] = base + a; S.h_e[hk] = e[a]; S.h_g[hk] = g[a]; S.h_p[hk] = prun; ++hk; }
    }
    if (tid == kSeqThreads - 1) { S.e_carry = e[PT - 1]; S.g_carry = g[PT - 1]; }
    if (tid == 0) S.nheads = htot;
    __syncthreads();
    // segment minima / maxima of P over the non-head terms (a thread's terms are consecutive: one flush per segment run)
    {
        int seg = hbase - 1;
        long long mn = LLONG_MAX, mx = LLONG_MIN;
#pragma unroll
        for (int a = 0; a < PT; ++a) {
            const int j = base + a;
            if (j >= cnt) break;
            if (hd[a]) {
                if (seg >= 0 && mn != LLONG_MAX) { atomicMin(&S.h_min[seg], mn); atomicMax(&S.h_max[seg], mx); }
                ++seg;
                mn = LLONG_MAX;
                mx = LLONG_MIN;
                continue;
            }
            if (seg < 0) continue;                               // zeros before the first head
            mn = P[a] < mn ? P[a] : mn;
            mx = P[a] > mx ? P[a] : mx;
        }
        if (seg >= 0 && mn != LLONG_MAX) { atomicMin(&S.h_min[seg], mn); atomicMax(&S.h_max[seg], mx); }
    }
    __syncthreads();
    if (wid == 0) {
        float s = s_in;
        int fbs = 0;
        for (int k0 = 0; k0 < htot; k0 += 64) {
            const int kk = k0 + lane;
            int hi = 0, he = 0, hg = 0, hend = cnt;
            long long hp = 0, pend = ptot, hmn = LLONG_MAX, hmx = LLONG_MIN;
            float hx = 0.0f;
            if (kk < htot) {
                hi = S.h_idx[kk];
                he = S.h_e[kk];
                hg = S.h_g[kk];
                hp = S.h_p[kk];
                hmn = S.h_min[kk];
                hmx = S.h_max[kk];
                hx = s_x[hi];
                if (kk + 1 < htot) { pend = S.h_p[kk + 1]; hend = S.h_idx[kk + 1]; }
            }
            const int m = min(64, htot - k0);
            for (int l = 0; l < m; ++l) {
                const int h = __builtin_amdgcn_readlane(hi, l), end = __builtin_amdgcn_readlane(hend, l);
                s = s + __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, hx), l));
                if (end > h + 1) {
                    const int E = __builtin_amdgcn_readlane(he, l), G = __builtin_amdgcn_readlane(hg, l);
                    const long long p0 = rl64i(hp, l);
                    const long long lo_q = rl64i(hmn, l) - p0, hi_q = rl64i(hmx, l) - p0, Q = rl64i(pend, l) - p0;
                    const double d = static_cast<double>(s);
                    const double u = ldexp(1.0, E - 23);
                    const double lo = ldexp(1.0, E) + u, top = ldexp(1.0, E + 1) - u;
                    bool ok = binade_abs(d) == E && E != kExpNone && (G > 0 ? d > 0.0 : d < 0.0) &&
                              rl64i(hmn, l) != LLONG_MAX;
                    if (ok) {
                        const double a0 = d + static_cast<double>(lo_q) * u, a1 = d + static_cast<double>(hi_q) * u;
                        ok = G > 0 ? (a0 >= lo && a1 <= top) : (-a1 >= lo && -a0 <= top);
                    }
                    if (ok) {
                        s = static_cast<float>(d + static_cast<double>(Q) * u);
                    } else {
                        for (int j = h + 1; j < end; ++j) s = s + s_x[j];
                        ++fbs;
                    }
                }
            }
        }
        if (lane == 0) { S.result = s; S.fb_seg = fbs; }
    }
    __syncthreads();
    s_out = S.result;
    T_out = T0 + ttot;
    e_out = S.e_carry;
    g_out = S.g_carry;
    return true;
}

}  // namespace lo
