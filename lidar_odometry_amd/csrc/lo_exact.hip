// lo_exact.hip — reference-exact GN step (lo_set_exact): the reference's own fp32 arithmetic order where the fast
// path reorders it.  IterativeClosestPointOptimizer.cpp:304-449 sums H, g and the cost SEQUENTIALLY in fp32 over the
// correspondences in scan order, takes the iteration-0 scale from the SORTED residuals, solves with Eigen's fp32 LDLT
// and re-projects SO3::Exp and the pose product through SO3(Matrix3f)'s JacobiSVD (MathUtils.cpp:23-39, :86-99).
// The fast path (lo_kernels.hip / lo_pko.hip) sums in fixed-order trees with fp64 block partials, merges the scale
// by Chan's formula and solves in fp64 with a Newton polar factor -- within 1e-7 of these, but not bit-equal, and over
// long GN sequences such ~1e-7 differences can move a correspondence across a voxel face.  Here every operation is
// the oracle's restatement (oracle/src/lo_oracle.cpp build_ne / iter0_scale / ldlt6_solve / so3_exp / se3_mul),
// so a scan's per-iteration logs equal the oracle's bit for bit (tests/test_gpu_exact.py).  It costs a sequential
// sum per iteration (~15 us at KITTI size) and two fp32 Jacobi SVDs per solve: a parity mode, not the default.
// Scans up to kExactMaxPoints (the sort and the term buffer are sized for it).
#include <algorithm>
#include <cfloat>

#include "lo_device.h"
#include "lo_math.h"
#include "lo_seqsum.h"
#include "lo_exact.h"

namespace lo {

// Diagnostic build only (-DLO_EXACT_STAMPS, `make diag`): thread 0 of the scale kernel stores s_memtime at its phase
// boundaries into DevState::dbg (lo_debug_counters); the product kernel executes no stamp.
#ifdef LO_EXACT_STAMPS
#define LO_XSTAMP(st, i) do { if (threadIdx.x == 0) (st)->dbg[i] = __builtin_amdgcn_s_memtime(); } while (0)
#define LO_XSTAT(st, i, v) do { if (threadIdx.x == 0) (st)->dbg[i] = static_cast<unsigned long long>(v); } while (0)
#else
#define LO_XSTAMP(st, i) do { } while (0)
#define LO_XSTAT(st, i, v) do { } while (0)
#endif

// ---- iteration 0: scale = sqrt(var) / 6 of the residuals sorted ascending, mean and variance summed in that order
// (IterativeClosestPointOptimizer.cpp:304-316).  One workgroup: the accepted residuals (+inf for the rest) sorted in
// registers / LDS (bitonic, lo_seqsum.h), then both sequential sums reproduced by mono_seq_sum (integer prefix sums
// between binade changes, a short walk over the segment heads) -- the same bits as std::accumulate's chain ----

// The sort is a rank computation spread over the chip (one KITTI scan's 4k residuals keep one CU busy for ~40 us in a
// bitonic network, VALU-bound): k_rank_sort gives every residual its rank -- #{smaller} + #{equal and earlier} on the
// fp64 bit patterns (non-negative doubles order as their bits; +inf marks a point without a correspondence, NaN sorts
// after it) -- with a wave per residual comparing it against the keys staged in LDS, and scatters it to that rank.
// The compares are latency-bound, so the grid is wide (n/4 workgroups of 32 KB LDS, ~4 waves per SIMD at 4k points).
constexpr int kRankTPE = 64;                                   // lanes per residual
constexpr int kRankThreads = 256;
constexpr int kRankStage = 4096;                               // keys staged per pass (32 KB of LDS)
// A residual's sort key: its fp64 bits, +inf for a point without a correspondence or past the scan.  Branch-free with
// clamped indices, so the staging loop's loads all go out together.
template <bool RAW>
__device__ __forceinline__ uint64_t rank_key(const int32_t* __restrict__ slot, const double* __restrict__ res, int n, int i) {
    constexpr uint64_t kInfBits = 0x7FF0000000000000ull;
    const int ic = i < n ? i : 0;
    const uint64_t r = static_cast<uint64_t>(__double_as_longlong(res[ic]));
    if constexpr (RAW) return i < n ? r : kInfBits;
    const int s = slot[ic];
    return (i < n && s >= 0) ? r : kInfBits;
}
template <bool RAW>
__global__ __launch_bounds__(kRankThreads) void k_rank_sort(KParams P, const double* raw, int n_raw, int n2, double* out) {
    if (!RAW && P.st->done) return;
    __shared__ uint64_t s_k[kRankStage];
    if (!RAW && blockIdx.x == 0) LO_XSTAMP(P.st, 5);
    const int tid = threadIdx.x, sub = tid & (kRankTPE - 1);
    const int el = blockIdx.x * (kRankThreads / kRankTPE) + tid / kRankTPE;
    const int n = RAW ? n_raw : scan_n(P);
    const int32_t* slot = P.slot;
    const double* res = RAW ? raw : (P.kd_res ? P.kd_res : P.res_out);
    const uint64_t ke = el < n2 ? rank_key<RAW>(slot, res, n, el) : ~0ull;
    int cnt = 0;
    for (int s0 = 0; s0 < n2; s0 += kRankStage) {
        const int m = min(kRankStage, n2 - s0);
        __syncthreads();
        for (int t0 = 0; t0 < m; t0 += 8 * kRankThreads) {   // eight keys' loads in flight per thread
            uint64_t kk[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) kk[u] = rank_key<RAW>(slot, res, n, s0 + t0 + u * kRankThreads + tid);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int t = t0 + u * kRankThreads + tid;
                if (t < m) s_k[t] = kk[u];
            }
        }
        __syncthreads();
        if (!RAW && blockIdx.x == 0) LO_XSTAMP(P.st, 6);
        for (int j0 = 0; j0 < m; j0 += 8 * kRankTPE) {     // eight LDS reads in flight, then the compares
            uint64_t kj[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) kj[u] = s_k[min(j0 + u * kRankTPE + sub, m - 1)];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = j0 + u * kRankTPE + sub;
                cnt += (j < m && (kj[u] < ke || (kj[u] == ke && s0 + j < el))) ? 1 : 0;
            }
        }
    }
    if (!RAW && blockIdx.x == 0) LO_XSTAMP(P.st, 7);
#pragma unroll
    for (int o = 1; o < kRankTPE; o <<= 1) cnt += __shfl_xor(cnt, o, kRankTPE);
    if (sub == 0 && el < n2) out[cnt] = __longlong_as_double(static_cast<long long>(ke));
}

template <int PT>
__global__ __launch_bounds__(kSeqThreads) void k_exact_scale(KParams P, const double* __restrict__ sorted) {
    DevState* st = P.st;
    if (st->done) return;
    extern __shared__ double s_x[];                          // kSeqThreads * PT doubles
    __shared__ SeqScratch S;
    LO_XSTAMP(st, 0);
    const int tid = threadIdx.x, base = tid * PT;
    // the accepted residuals are the sorted array's finite entries (the rest are the +inf of points without a
    // correspondence and the padding; a NaN residual sorts after them)
    int nacc = 0;
    double v[PT];
    bool nan = false;
#pragma unroll
    for (int a = 0; a < PT; ++a) {
        v[a] = sorted[base + a];
        nan = nan || isnan(v[a]);
        nacc += (v[a] != __builtin_inf() && !isnan(v[a])) ? 1 : 0;
    }
    int cnt;
    (void)block_excl_scan<int>(nacc, S.wi, cnt);
    const bool any_nan = __syncthreads_or(nan ? 1 : 0) != 0;
    if (cnt == 0) return;                                    // too few correspondences: the PKO launch reports it
    if (any_nan) {                                           // a NaN residual: mean, variance and scale are NaN
        if (nan) st->scale = sqrt(v[0] + v[PT - 1]) / 6.0;
        return;
    }
    LO_XSTAMP(st, 1);
#pragma unroll
    for (int a = 0; a < PT; ++a) s_x[base + a] = v[a];
    __syncthreads();
    LO_XSTAMP(st, 2);
    double sum;
    if (!mono_seq_sum<PT>(cnt, s_x, S, 0.0, kExpNone, false, 0.0, sum)) sum = chain_seq_sum(s_x, cnt, 0.0, S);
    LO_XSTAMP(st, 3);
    LO_XSTAT(st, 8, S.nheads);
    LO_XSTAT(st, 9, S.fb_seg);
    LO_XSTAT(st, 10, S.fb_terms);
    LO_XSTAT(st, 14, cnt);
    const double mean = sum / cnt;
    double w[PT];
#pragma unroll
    for (int a = 0; a < PT; ++a) {
        w[a] = (base + a < cnt) ? (v[a] - mean) * (v[a] - mean) : 0.0;
        s_x[base + a] = w[a];
    }
    __syncthreads();
    double var;
    if (!mono_seq_sum<PT>(cnt, s_x, S, 0.0, kExpNone, false, 0.0, var)) var = chain_seq_sum(s_x, cnt, 0.0, S);
    LO_XSTAMP(st, 4);
    LO_XSTAT(st, 11, S.nheads);
    LO_XSTAT(st, 12, S.fb_seg);
    LO_XSTAT(st, 13, S.fb_terms);
    var /= cnt;
    if (tid == 0) st->scale = sqrt(var) / 6.0;
}

// ---- iteration 0 for scans beyond the one-workgroup sort (kExactMaxPoints < n): k_exact_resid writes every point's
// residual (+inf without a correspondence) to global memory, the context sorts them ascending (hipCUB radix sort:
// the same order as std::sort for the non-NaN values; -0 / +0 ties do not change any sum), and k_exact_scale_g
// runs both sequential sums over the sorted residuals chunk by chunk (mono_seq_sum with the prediction and the running
// sum carried from chunk to chunk; every chunk starts a segment) ----
__global__ __launch_bounds__(kBlock) void k_exact_resid(KParams P, double* out) {
    DevState* st = P.st;
    const int i = blockIdx.x * kBlock + threadIdx.x, n = scan_n(P);
    if (i >= P.n) return;
    double v = __builtin_inf();                                // also past a device-counted scan's end (sorted last)
    const int s = i < n ? P.slot[i] : -1;
    if (s >= 0 && P.kd_res) {
        v = P.kd_res[i];
    } else if (s >= 0) {
        float T[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
        float wx, wy, wz;
        transform_pt(T, P.pts[3 * i], P.pts[3 * i + 1], P.pts[3 * i + 2], wx, wy, wz);
        v = residual_f64(P.tab[s], wx, wy, wz);
    }
    out[i] = v;
}

constexpr int kScaleGPT = 8;
constexpr int kScaleGChunk = kSeqThreads * kScaleGPT;          // terms per chunk (64 KB of LDS)
template <bool SQ>
__device__ __forceinline__ double chunked_seq_sum(const double* __restrict__ x, int cnt, double m, double* s_x, SeqScratch& S) {
    const int tid = threadIdx.x;
    double s = 0.0, Tc = 0.0;
    int ec = kExpNone;
    for (int c0 = 0; c0 < cnt; c0 += kScaleGChunk) {
        const int mc = min(kScaleGChunk, cnt - c0);
        for (int k = tid; k < kScaleGChunk; k += kSeqThreads) {
            double v = 0.0;
            if (k < mc) {
                v = x[c0 + k];
                if constexpr (SQ) v = (v - m) * (v - m);
            }
            s_x[k] = v;
        }
        __syncthreads();
        if (mono_seq_sum<kScaleGPT>(mc, s_x, S, Tc, ec, true, s, s)) ec = S.e_carry;
        else { s = chain_seq_sum(s_x, mc, s, S); ec = binade64(s); }
        Tc = s;                                                // the exact running sum predicts the next chunk best
        __syncthreads();                                       // s_x / S reuse by the next chunk
    }
    return s;
}
__global__ __launch_bounds__(kSeqThreads) void k_exact_scale_g(KParams P, const double* __restrict__ sorted) {
    DevState* st = P.st;
    if (st->done) return;
    __shared__ double s_x[kScaleGChunk];
    __shared__ SeqScratch S;
    __shared__ int s_cnt;
    const int tid = threadIdx.x, n = scan_n(P);
    if (tid == 0) s_cnt = n;
    __syncthreads();
    int nan = 0;
    for (int i = tid; i < n; i += kSeqThreads) {
        const double v = sorted[i];
        if (v == __builtin_inf() && (i == 0 || sorted[i - 1] != __builtin_inf())) atomicMin(&s_cnt, i);
        nan |= isnan(v) ? 1 : 0;
    }
    const bool any_nan = __syncthreads_or(nan) != 0;
    const int cnt = s_cnt;
    if (cnt == 0) return;                                      // too few correspondences: the PKO launch reports it
    if (any_nan) {
        if (tid == 0) {
            double s = 0.0;
            for (int i = 0; i < n; ++i) if (sorted[i] != __builtin_inf()) s = s + sorted[i];
            st->scale = sqrt(s) / 6.0;
        }
        return;
    }
    const double sum = chunked_seq_sum<false>(sorted, cnt, 0.0, s_x, S);
    const double var = chunked_seq_sum<true>(sorted, cnt, sum / cnt, s_x, S);
    if (tid == 0) st->scale = sqrt(var / cnt) / 6.0;
}

// Parity / diagnostic entry (lo_seq_sum_f64): the sequential sum of n <= kExactMaxPoints non-negative doubles in
// index order (sorted ascending first with SORT), by the same sort and mono_seq_sum as k_exact_scale.  out[0] = the
// sum; stats = heads, fallback segments, fallback terms, s_memtime cycles of the sort + sum.
template <int PT>
__global__ __launch_bounds__(kSeqThreads) void k_seq_sum_diag(const double* __restrict__ x, int n, double* out,
                                                             long long* stats) {
    extern __shared__ double s_x[];
    __shared__ SeqScratch S;
    const int tid = threadIdx.x, base = tid * PT;
    double v[PT];
#pragma unroll
    for (int a = 0; a < PT; ++a) v[a] = (base + a < n) ? x[base + a] : 0.0;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int a = 0; a < PT; ++a) s_x[base + a] = v[a];
    __syncthreads();
    double sum;
    long long heads = -1;                                    // -1: more than kSeqHeadCap heads (the plain chain ran)
    if (tid == 0) S.fb_seg = S.fb_terms = 0;
    if (mono_seq_sum<PT>(n, s_x, S, 0.0, kExpNone, false, 0.0, sum)) heads = S.nheads;
    else sum = chain_seq_sum(s_x, n, 0.0, S);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) {
        out[0] = sum;
        stats[0] = heads;
        stats[1] = S.fb_seg;
        stats[2] = S.fb_terms;
        stats[3] = static_cast<long long>(t1 - t0);
    }
}
template <int PT>
static void launch_seq_diag_pt(const double* x, int n, double* out, long long* stats, hipStream_t s) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_seq_sum_diag<PT>), hipFuncAttributeMaxDynamicSharedMemorySize,
                              kSeqThreads * PT * 8);
    hipLaunchKernelGGL(k_seq_sum_diag<PT>, dim3(1), dim3(kSeqThreads), static_cast<size_t>(kSeqThreads) * PT * 8, s, x, n,
                       out, stats);
}
// sort (nullable scratch of n doubles): the values ranked and scattered by k_rank_sort first, as the exact scale does
void launch_seq_sum_diag(const double* x, int n, double* sort, double* out, long long* stats, hipStream_t s) {
    const double* src = x;
    if (sort) {
        KParams P{};
        if (n > 0)
            hipLaunchKernelGGL(k_rank_sort<true>, dim3((n + kRankThreads / kRankTPE - 1) / (kRankThreads / kRankTPE)),
                               dim3(kRankThreads), 0, s, P, x, n, n, sort);
        src = sort;
    }
    if (n <= kSeqThreads) launch_seq_diag_pt<1>(src, n, out, stats, s);
    else if (n <= 2 * kSeqThreads) launch_seq_diag_pt<2>(src, n, out, stats, s);
    else if (n <= 4 * kSeqThreads) launch_seq_diag_pt<4>(src, n, out, stats, s);
    else if (n <= 8 * kSeqThreads) launch_seq_diag_pt<8>(src, n, out, stats, s);
    else launch_seq_diag_pt<16>(src, n, out, stats, s);
}

// Host side: the scale of a scan of at most kExactMaxPoints points: k_rank_sort into `sorted` (n doubles of scratch),
// then k_exact_scale<PT> (PT = the padded size / kSeqThreads).
template <int PT>
static void launch_scale_pt(const KParams& P, const double* sorted, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_exact_scale<PT>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kSeqThreads * PT * 8);
        attr = true;
    }
    hipLaunchKernelGGL(k_exact_scale<PT>, dim3(1), dim3(kSeqThreads), static_cast<size_t>(kSeqThreads) * PT * 8, s, P,
                       sorted);
}
void launch_exact_scale(const KParams& P, int n, double* sorted, hipStream_t s) {
    int PT = std::max(1, (n + kSeqThreads - 1) / kSeqThreads);
    PT = PT <= 8 ? PT : (PT <= 10 ? 10 : (PT <= 12 ? 12 : 16));   // the instantiated widths
    const int n2 = PT * kSeqThreads;                         // padded: ranks of the +inf padding fill [n, n2)
    hipLaunchKernelGGL(k_rank_sort<false>, dim3(n2 / (kRankThreads / kRankTPE)), dim3(kRankThreads), 0, s, P,
                       static_cast<const double*>(nullptr), 0, n2, sorted);
    switch (PT) {
        case 1: launch_scale_pt<1>(P, sorted, s); break;
        case 2: launch_scale_pt<2>(P, sorted, s); break;
        case 3: launch_scale_pt<3>(P, sorted, s); break;
        case 4: launch_scale_pt<4>(P, sorted, s); break;
        case 5: launch_scale_pt<5>(P, sorted, s); break;
        case 6: launch_scale_pt<6>(P, sorted, s); break;
        case 7: launch_scale_pt<7>(P, sorted, s); break;
        case 8: launch_scale_pt<8>(P, sorted, s); break;
        case 10: launch_scale_pt<10>(P, sorted, s); break;
        case 12: launch_scale_pt<12>(P, sorted, s); break;
        default: launch_scale_pt<16>(P, sorted, s); break;
    }
}

// ---- per-correspondence terms of build_ne (:345-410) with this iteration's Huber delta: H[row][col] =
// J[col] * (w J[row]) (all 36), g[j] = (w r) J[j], cost = (w r) r; zeros for points without a correspondence
// (adding +0 to the running sums leaves them unchanged) ----
__global__ __launch_bounds__(kBlock) void k_exact_terms(KParams P) {
    DevState* st = P.st;
    if (st->done) return;
    __shared__ double s_alpha;
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid < kWave) {
        const double a = P.use_pko ? pko_select_alpha(P) : P.robust_delta;
        if (lane == 0) {
            s_alpha = a;
            if (blockIdx.x == 0) st->alpha = a;
        }
    }
    __syncthreads();
    const int i = blockIdx.x * kBlock + tid;
    if (i >= scan_n(P)) return;
    // row-major [point][43], or term-major [43][ex_ld] (coalesced columns for k_exact_sum43)
    const size_t o0 = P.ex_ld ? static_cast<size_t>(i) : static_cast<size_t>(i) * kExactTerms;
    const size_t os = P.ex_ld ? static_cast<size_t>(P.ex_ld) : 1;
    float* out = P.ex_terms + o0;
    const int s = P.slot[i];
    if (s < 0) {
        for (int k = 0; k < kExactTerms; ++k) out[k * os] = 0.0f;
        return;
    }
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
    const double scale = st->scale;
    const float dl = static_cast<float>(s_alpha);
    const float px = P.pts[3 * i], py = P.pts[3 * i + 1], pz = P.pts[3 * i + 2];
    const Slot sl = P.tab[s];
    double r64;
    if (P.kd_res) {
        r64 = P.kd_res[i];
    } else {
        float wx, wy, wz;
        transform_pt(T, px, py, pz, wx, wy, wz);
        r64 = residual_f64(sl, wx, wy, wz);
    }
    float f[14];
    exact_point_factors(P, T, scale, dl, r64, px, py, pz, sl, f);
    for (int k = 0; k < kExactTerms; ++k) {
        int fa, fb;
        exact_term_factors(k, fa, fb);
        out[k * os] = f[fa] * f[fb];
    }
}

// ---- the running fp32 sums over the correspondences in scan order (one lane per H / g / cost entry), then the
// reference's solve and right-update, convergence test and the iteration's log ----
// The 43 sums run in point order, one lane each (wave 0), over the term rows staged through LDS: the other waves
// copy chunk c + 1 (contiguous in the row-major term buffer, so coalesced) while wave 0 sums chunk c, so the
// sequential adds wait on LDS rather than on a global round trip per row (one lane loading its column from global
// memory, 8 rows in flight, took ~140 us at KITTI size).
constexpr int kExactSolveThreads = 512;
constexpr int kExactRows = 160;                                // rows per chunk; 2 chunks x 27.5 KB of LDS
constexpr int kExactChunk = kExactRows * kExactTerms;
constexpr int kExactPer = (kExactChunk + kExactSolveThreads - kWave - 1) / (kExactSolveThreads - kWave);
__global__ __launch_bounds__(kExactSolveThreads) void k_exact_solve(KParams P, int it) {
    DevState* st = P.st;
    if (st->done) return;
    __shared__ float tot[kExactTerms];
    __shared__ float buf[2][kExactChunk];
    const int tid = threadIdx.x, lane = tid, n = scan_n(P);
    const int n_chunks = (n + kExactRows - 1) / kExactRows;
    const size_t total = static_cast<size_t>(n) * kExactTerms;
    for (int k = tid; k < kExactChunk && k < static_cast<int>(total); k += kExactSolveThreads) buf[0][k] = P.ex_terms[k];
    __syncthreads();
    float s = 0.0f;
    for (int c = 0; c < n_chunks; ++c) {
        if (tid >= kWave) {                                    // copy chunk c + 1 into the other buffer
            const size_t base = static_cast<size_t>(c + 1) * kExactChunk;
            float v[kExactPer];
#pragma unroll
            for (int u = 0; u < kExactPer; ++u) {
                const int k = (tid - kWave) + u * (kExactSolveThreads - kWave);
                v[u] = (k < kExactChunk && base + k < total) ? P.ex_terms[base + k] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < kExactPer; ++u) {
                const int k = (tid - kWave) + u * (kExactSolveThreads - kWave);
                if (k < kExactChunk) buf[(c + 1) & 1][k] = v[u];
            }
        } else if (lane < kExactTerms) {                       // the adds, in point order
            const float* rows = buf[c & 1] + lane;
            const int m = min(kExactRows, n - c * kExactRows);
            int r = 0;
            for (; r + 16 <= m; r += 16) {
                float v[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) v[u] = rows[(r + u) * kExactTerms];
#pragma unroll
                for (int u = 0; u < 16; ++u) s += v[u];
            }
            for (; r < m; ++r) s += rows[r * kExactTerms];
        }
        __syncthreads();
    }
    if (lane < kExactTerms) tot[lane] = s;
    __syncthreads();
    if (lane != 0) return;
    float tf[kExactTerms], pn[12], delta[6];
    for (int k = 0; k < kExactTerms; ++k) tf[k] = tot[k];
    const bool conv = exact_solve_step(tf, st->pose, P.tol_t, P.tol_r, pn, delta);
    for (int q = 0; q < 12; ++q) st->pose[q] = pn[q];
    if (it < LO_MAX_ITERS) {
        lo_iter_log& L = st->logs[it];
        for (int q = 0; q < 12; ++q) L.pose[q] = pn[q];
        L.n_corr = st->n_corr;
        L.scale = st->scale;
        L.alpha = st->alpha;
        L.cost = tot[42];
        int k = 0;
        for (int r = 0; r < 6; ++r) for (int c = r; c < 6; ++c) L.H[k++] = tot[r * 6 + c];
        for (int j = 0; j < 6; ++j) { L.g[j] = tot[36 + j]; L.delta[j] = delta[j]; }
    }
    st->iter = it + 1;
    if (conv) st->done = 1;
}

// ---- large scans (n > kExactMaxPoints): the 43 running sums of build_ne in point order, one workgroup per term
// column of the term-major buffer, each reproduced by signed_seq_sum (lo_seqsum.h: integer prefix sums between the
// running sum's predicted binade / sign changes) chunk by chunk; k_exact_finish then solves as k_exact_solve does ----
constexpr int kSumPT = 4;
constexpr int kSumChunk = kSeqThreads * kSumPT;
// col[0, n) summed in fp32 in index order, as the reference's running sums do; stats (nullable): heads, segments
// summed term by term, chunks that fell back to the plain chain.
__device__ __forceinline__ float column_seq_sum(const float* __restrict__ col, int n, float* s_x, SeqScratchS& S, int* stats) {
    const int tid = threadIdx.x;
    float s = 0.0f;
    int ec = kExpNone, gc = 0, nh = 0, fb = 0, chains = 0;
    for (int c0 = 0; c0 < n; c0 += kSumChunk) {
        const int mc = min(kSumChunk, n - c0);
        for (int t = tid; t < kSumChunk; t += kSeqThreads) s_x[t] = t < mc ? col[c0 + t] : 0.0f;
        __syncthreads();
        int en, gn;
        if (signed_seq_sum<kSumPT>(mc, s_x, S, static_cast<double>(s), ec, gc, s, s, en, gn)) {
            nh += S.nheads;
            fb += S.fb_seg;
        } else {
            if (tid < kWave) {                                 // more heads than the list holds: the plain chain
                for (int j = 0; j < mc; ++j) s = s + s_x[j];
                if (tid == 0) S.result = s;
            }
            __syncthreads();
            s = S.result;
            en = binade_abs(static_cast<double>(s));
            gn = s > 0.0f ? 1 : (s < 0.0f ? -1 : 0);
            ++chains;
        }
        ec = en;
        gc = gn;
        __syncthreads();                                       // s_x / S reuse by the next chunk
    }
    if (stats && tid == 0) { stats[0] = nh; stats[1] = fb; stats[2] = chains; }
    return s;
}
__global__ __launch_bounds__(kSeqThreads) void k_exact_sum43(KParams P) {
    DevState* st = P.st;
    if (st->done) return;
    __shared__ float s_x[kSumChunk];
    __shared__ SeqScratchS S;
    const float s = column_seq_sum(P.ex_terms + static_cast<size_t>(blockIdx.x) * P.ex_ld, scan_n(P), s_x, S, nullptr);
    if (threadIdx.x == 0) P.ex_tot[blockIdx.x] = s;
}
// Parity / diagnostic entry (lo_seq_sum_f32): one column through the same reproduction.
__global__ __launch_bounds__(kSeqThreads) void k_seq_sum_f32_diag(const float* __restrict__ x, int n, float* out,
                                                                  long long* stats) {
    __shared__ float s_x[kSumChunk];
    __shared__ SeqScratchS S;
    __shared__ int st3[3];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const float s = column_seq_sum(x, n, s_x, S, st3);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (threadIdx.x == 0) {
        out[0] = s;
        stats[0] = st3[0];
        stats[1] = st3[1];
        stats[2] = st3[2];
        stats[3] = static_cast<long long>(t1 - t0);
    }
}
void launch_seq_sum_f32_diag(const float* x, int n, float* out, long long* stats, hipStream_t s) {
    hipLaunchKernelGGL(k_seq_sum_f32_diag, dim3(1), dim3(kSeqThreads), 0, s, x, n, out, stats);
}

__global__ void k_exact_finish(KParams P, int it) {
    DevState* st = P.st;
    if (st->done || threadIdx.x != 0) return;
    float tot[kExactTerms], pn[12], delta[6];
    for (int k = 0; k < kExactTerms; ++k) tot[k] = P.ex_tot[k];
    const bool conv = exact_solve_step(tot, st->pose, P.tol_t, P.tol_r, pn, delta);
    for (int q = 0; q < 12; ++q) st->pose[q] = pn[q];
    if (it < LO_MAX_ITERS) {
        lo_iter_log& L = st->logs[it];
        for (int q = 0; q < 12; ++q) L.pose[q] = pn[q];
        L.n_corr = st->n_corr;
        L.scale = st->scale;
        L.alpha = st->alpha;
        L.cost = tot[42];
        int k = 0;
        for (int r = 0; r < 6; ++r) for (int c = r; c < 6; ++c) L.H[k++] = tot[r * 6 + c];
        for (int j = 0; j < 6; ++j) { L.g[j] = tot[36 + j]; L.delta[j] = delta[j]; }
    }
    st->iter = it + 1;
    if (conv) st->done = 1;
}

}  // namespace lo
