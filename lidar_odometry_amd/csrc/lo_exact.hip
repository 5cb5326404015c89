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

#include "lo_blocksort.h"
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

// ---- iteration 0, scans of at most kExactMergeMax points: the correspondence launch left one sorted run of 256 keys per
// block (presort_block, lo_blocksort.h).  k_rank_runs (one workgroup per run, every run staged in LDS) places each key
// at its rank -- its position in its own run plus, in every other run, the keys below it (later runs) or not above it
// (earlier runs): nine probes per run, the runs' searches interleaved -- and k_exact_scale_s sums the sorted array in
// one workgroup (mono_sum_tx: the halfway ties as two-state segment maps, a walk over ~25 binade heads). ----
__global__ __launch_bounds__(kBlock) void k_rank_runs(KParams P, const uint64_t* __restrict__ runs, uint64_t* __restrict__ out) {
    if (P.st->done) return;
    if (blockIdx.x == 0) LO_XSTAMP(P.st, 15);
    extern __shared__ uint64_t s_r[];                        // P.nb runs
    const int nb = P.nb, b = blockIdx.x, tid = threadIdx.x;
    {                                                        // every run's key of this lane in flight at once
        constexpr int kRuns = kExactMergeMax / kBlock;
        uint64_t v[kRuns];
#pragma unroll
        for (int r = 0; r < kRuns; ++r) v[r] = runs[(r < nb ? r : 0) * kBlock + tid];
#pragma unroll
        for (int r = 0; r < kRuns; ++r) if (r < nb) s_r[r * kBlock + tid] = v[r];
    }
    __syncthreads();
    if (b == 0) LO_XSTAMP(P.st, 12);
    const uint64_t x = s_r[b * kBlock + tid];
    // equal keys: earlier runs first, then this run's order
    const int rank = tid + (nb <= 16 ? runs_rank<16>(s_r, nb, b, x) : runs_rank<kExactMergeMax / kBlock>(s_r, nb, b, x));
    out[rank] = x;
    if (b == 0) LO_XSTAMP(P.st, 13);
}

template <int NT, int PT>
__global__ __launch_bounds__(NT) void k_exact_scale_s(KParams P, const uint64_t* __restrict__ sorted) {
    DevState* st = P.st;
    if (st->done) return;
    extern __shared__ double s_x[];                          // NT * PT terms
    __shared__ MonoScratch<NT> S;
    __shared__ int s_cnt[NT / kWave];
    LO_XSTAMP(st, 0);
    const int tid = threadIdx.x, base = tid * PT;
    const int nfill = P.nb * kBlock;                         // sorted keys (finite residuals first, then +inf / NaN)
    uint64_t v[PT];
#pragma unroll
    for (int q = 0; q < PT; ++q) v[q] = base + q < nfill ? sorted[base + q] : kInfKey;
    // accepted residuals = the finite keys (a prefix); a NaN residual (accepted: the gate keeps NaN) makes the mean,
    // the variance and the scale NaN
    int nacc = 0;
    bool nan = false;
    uint64_t nan_key = 0;
#pragma unroll
    for (int q = 0; q < PT; ++q) {
        nacc += v[q] < kInfKey ? 1 : 0;
        if (v[q] > kInfKey && !nan) { nan = true; nan_key = v[q]; }
    }
    int cnt = 0;
    (void)block_excl_scan_dpp<NT>(nacc, 0, [](int a, int c) { return a + c; }, s_cnt, &cnt);
    const bool any_nan = __syncthreads_or(nan ? 1 : 0) != 0;
    if (cnt == 0) return;                                    // too few correspondences: the PKO launch reports it
    if (any_nan) {
        if (nan) st->scale = sqrt(__longlong_as_double(static_cast<long long>(nan_key))) / 6.0;
        return;
    }
    double x[PT];
#pragma unroll
    for (int q = 0; q < PT; ++q) {
        x[q] = base + q < cnt ? __longlong_as_double(static_cast<long long>(v[q])) : 0.0;
        s_x[base + q] = x[q];
    }
    __syncthreads();
    LO_XSTAMP(st, 1);
#ifdef LO_EXACT_STAMPS
    unsigned long long* stp = st->dbg + 4;                  // dbg[4..6]: the mean sum's phases
    {                                                        // diagnostic: the same sum once more from a warm
        double warm;                                         // instruction cache (dbg[8..10] phases, dbg[11] end)
        LO_XSTAMP(st, 7);
        (void)mono_sum_tx<NT, PT>(x, cnt, s_x, S, warm, st->dbg + 8);
        LO_XSTAMP(st, 11);
    }
#else
    unsigned long long* stp = nullptr;
#endif
    double sum;
    if (!mono_sum_tx<NT, PT>(x, cnt, s_x, S, sum, stp)) sum = chain_sum_tx<NT>(s_x, cnt, S);
    LO_XSTAMP(st, 2);
    LO_XSTAT(st, 14, cnt);
    const double mean = sum / cnt;                           // std::accumulate(...) / residuals.size()
#pragma unroll
    for (int q = 0; q < PT; ++q) {
        x[q] = base + q < cnt ? (x[q] - mean) * (x[q] - mean) : 0.0;
        s_x[base + q] = x[q];                                // the walk's reads of s_x ended at mono_sum_tx's barrier
    }
    __syncthreads();
    double var;
    if (!mono_sum_tx<NT, PT>(x, cnt, s_x, S, var)) var = chain_sum_tx<NT>(s_x, cnt, S);
    LO_XSTAMP(st, 3);
    var /= cnt;
    if (tid == 0) st->scale = sqrt(var) / 6.0;               // :313-315
}

// ---- iteration 0, scans of at most kExactMergeMax points, in ONE launch after the correspondence launch: the accepted
// residuals' keys sorted by a counting sort in LDS -- bins over [min, max] of the finite keys (monotone in the key, so
// bin order is sort order), a histogram, its scan, an atomic scatter into the bins, then each key's rank inside its
// bin by comparing it with the bin's members (a bin holds a few keys: the bins are as many as the keys) -- and both
// sums by mono_sum_tx.  No chip-wide pass, no presort. ----
struct KeyStat {
    uint64_t mn, mx;                                         // min / max finite key
    int cnt, nan;                                            // finite keys; NaN keys
};
__device__ __forceinline__ KeyStat keystat_op(KeyStat a, KeyStat b) {
    return KeyStat{a.mn < b.mn ? a.mn : b.mn, a.mx > b.mx ? a.mx : b.mx, a.cnt + b.cnt, a.nan | b.nan};
}
constexpr int kScaleC = 1024;                                // k_exact_scale_c threads
template <int PT>
__host__ __device__ constexpr int scale_c_bins() { return PT * kScaleC <= 4096 ? PT * kScaleC : (PT <= 8 ? 2048 : 1024); }
template <int PT>
__host__ __device__ constexpr size_t scale_c_lds() {
    return static_cast<size_t>(PT) * kScaleC * sizeof(uint64_t) + 2 * static_cast<size_t>(scale_c_bins<PT>()) * sizeof(int);
}

// n: the scan's point count (<= PT * kScaleC); s_dyn: scale_c_lds<PT>() bytes; S / s_ks: the caller's static LDS (one
// copy for every width the device-dispatching kernel inlines)
template <int PT>
__device__ __forceinline__ void exact_scale_c_body(const KParams& P, int n, uint64_t* s_dyn, MonoScratch<kScaleC>& S,
                                                   KeyStat* s_ks) {
    DevState* st = P.st;
    constexpr int NT = kScaleC, N = PT * NT, NB = scale_c_bins<PT>();
    uint64_t* s_tmp = s_dyn;                                 // keys in bin order, then sorted (in place)
    int* s_cnt = reinterpret_cast<int*>(s_dyn + N);          // per-bin count
    int* s_end = s_cnt + NB;                                 // per-bin start, then end (after the scatter)
    LO_XSTAMP(st, 0);
    const int tid = threadIdx.x;
#ifndef LO_EXACT_STAMPS
    if (tid == 0) st->dbg[23] = N;                           // the sort width this scan ran (lo_debug_counters_ex)
#endif
    const int32_t* slot = P.slot;
    const double* res = P.kd_res ? P.kd_res : P.res_out;
    // the keys, coalesced: element e = q NT + tid (the accepted residual's bits, else +inf)
    uint64_t key[PT];
#pragma unroll
    for (int q = 0; q < PT; ++q) {
        const int e = q * NT + tid, ec = e < n ? e : 0;
        const int sl = slot[ec];
        const uint64_t r = static_cast<uint64_t>(__double_as_longlong(res[ec]));
        key[q] = (e < n && sl >= 0) ? r : kInfKey;
    }
    KeyStat ks{~0ull, 0ull, 0, 0};
#pragma unroll
    for (int q = 0; q < PT; ++q) {
        if (key[q] < kInfKey) { ks.mn = key[q] < ks.mn ? key[q] : ks.mn; ks.mx = key[q] > ks.mx ? key[q] : ks.mx; ++ks.cnt; }
        if (key[q] > kInfKey) ks.nan = 1;
    }
    for (int b = tid; b < NB; b += NT) s_cnt[b] = 0;
    KeyStat tot;
    (void)block_excl_scan_dpp<NT>(ks, KeyStat{~0ull, 0ull, 0, 0}, keystat_op, s_ks, &tot);
    const int cnt = tot.cnt;
    LO_XSTAMP(st, 13);
    if (cnt == 0) return;                                    // too few correspondences: the PKO launch reports it
    if (tot.nan) {                                           // a NaN residual (accepted: the gate keeps NaN): the mean,
        uint64_t nk = ~0ull;                                 // the variance and the scale are NaN
#pragma unroll
        for (int q = 0; q < PT; ++q) if (key[q] > kInfKey && key[q] < nk) nk = key[q];
        if (nk != ~0ull) st->scale = sqrt(__longlong_as_double(static_cast<long long>(nk))) / 6.0;
        return;
    }
    const uint64_t range = tot.mx - tot.mn;
    const int bl = range ? 64 - __clzll(static_cast<long long>(range)) : 0;
    int lb = 0;
    while ((1 << (lb + 1)) <= NB) ++lb;                      // log2(NB)
    const int shift = bl > lb ? bl - lb : 0;
    auto bin_of = [&](uint64_t k) { return static_cast<int>((k - tot.mn) >> shift); };
    // histogram, its exclusive scan (NB / NT consecutive bins per thread), the scatter
#pragma unroll
    for (int q = 0; q < PT; ++q) if (key[q] < kInfKey) atomicAdd(&s_cnt[bin_of(key[q])], 1);
    __syncthreads();
    constexpr int BPT = NB / NT;
    int bsum = 0;
    for (int i = 0; i < BPT; ++i) bsum += s_cnt[tid * BPT + i];
    int bex = block_excl_scan_dpp<NT>(bsum, 0, [](int a, int b) { return a + b; }, S.wi);
    for (int i = 0; i < BPT; ++i) { s_end[tid * BPT + i] = bex; bex += s_cnt[tid * BPT + i]; }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PT; ++q)
        if (key[q] < kInfKey) s_tmp[atomicAdd(&s_end[bin_of(key[q])], 1)] = key[q];
    __syncthreads();
    LO_XSTAMP(st, 14);
    // each key's rank in its bin: the members below it, and the equal ones placed before it; every key is read before
    // any moves (the barrier), so the sorted order goes back into the same array
    uint64_t kk[PT];
    int pos[PT];
#pragma unroll
    for (int i = 0; i < PT; ++i) {
        const int p = tid + i * NT;
        pos[i] = -1;
        if (p < cnt) {
            const uint64_t k = s_tmp[p];
            const int b = bin_of(k), e = s_end[b], s0 = e - s_cnt[b];
            int r = 0;
            for (int q = s0; q < e; ++q) {
                const uint64_t o = s_tmp[q];
                r += (o < k || (o == k && q < p)) ? 1 : 0;
            }
            kk[i] = k;
            pos[i] = s0 + r;
        }
    }
    LO_XSTAMP(st, 15);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PT; ++i)
        if (pos[i] >= 0) s_tmp[pos[i]] = kk[i];
    __syncthreads();
    const uint64_t* s_srt = s_tmp;
    LO_XSTAMP(st, 12);
    double* s_x = reinterpret_cast<double*>(s_tmp);          // each thread overwrites only the keys it reads
    const int base = tid * PT;
    double x[PT];
#pragma unroll
    for (int q = 0; q < PT; ++q) {
        x[q] = base + q < cnt ? __longlong_as_double(static_cast<long long>(s_srt[base + q])) : 0.0;
        s_x[base + q] = x[q];
    }
    __syncthreads();
    LO_XSTAMP(st, 1);
    double sum, var;
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {                   // the mean's sum, then the variance's (same code)
#ifdef LO_EXACT_STAMPS
        unsigned long long* stp = st->dbg + (pass ? 8 : 4);  // dbg[4..6] / dbg[8..10]: the sums' phases
#else
        unsigned long long* stp = nullptr;
#endif
        double v;
        if (!mono_sum_tx<NT, PT>(x, cnt, s_x, S, v, stp)) v = chain_sum_tx<NT>(s_x, cnt, S);
        if (pass == 0) {
            LO_XSTAMP(st, 2);
            sum = v;
            const double mean = sum / cnt;                   // std::accumulate(...) / residuals.size()
#pragma unroll
            for (int q = 0; q < PT; ++q) {
                x[q] = base + q < cnt ? (x[q] - mean) * (x[q] - mean) : 0.0;
                s_x[base + q] = x[q];                        // the walk's reads of s_x ended at mono_sum_tx's barrier
            }
            __syncthreads();
        } else {
            var = v;
        }
    }
    (void)sum;
    LO_XSTAMP(st, 3);
    var /= cnt;
    if (tid == 0) st->scale = sqrt(var) / 6.0;               // :313-315
}
template <int PT>
__global__ __launch_bounds__(kScaleC) void k_exact_scale_c(KParams P) {
    if (P.st->done) return;
    extern __shared__ uint64_t s_dyn[];
    __shared__ MonoScratch<kScaleC> S;
    __shared__ KeyStat s_ks[kScaleC / kWave];
    exact_scale_c_body<PT>(P, scan_n(P), s_dyn, S, s_ks);
}
// Device counts beyond 8192 (a fine filter over a large raw scan; never at the bench sizes): the same counting sort of
// up to 16384 keys in LDS with the keys re-read from global memory in two register rounds (no 16-key arrays: the
// one-kernel-for-every-width form spilled ~1 KB per lane and took 46 instead of 23 us on the narrow paths), then both
// sums as the plain sequential chain (chain_sum_tx: the reference's own loop on one wave, ~0.15 ms) -- exact by
// construction, no scratch.
constexpr int kScaleWideNB = 1024;
constexpr size_t kScaleWideLds = static_cast<size_t>(16) * kScaleC * sizeof(uint64_t) + 2 * kScaleWideNB * sizeof(int);
__device__ __forceinline__ void exact_scale_c_wide(const KParams& P, int n, uint64_t* s_dyn, MonoScratch<kScaleC>& S,
                                                KeyStat* s_ks) {
    constexpr int NT = kScaleC, RT = 8, N = 2 * RT * NT, NB = kScaleWideNB;
    DevState* st = P.st;
    uint64_t* s_tmp = s_dyn;
    int* s_cnt = reinterpret_cast<int*>(s_dyn + N);
    int* s_end = s_cnt + NB;
    const int tid = threadIdx.x;
    if (tid == 0) st->dbg[23] = N;                           // the sort width this scan ran (lo_debug_counters_ex)
    const int32_t* slot = P.slot;
    const double* res = P.kd_res ? P.kd_res : P.res_out;
    auto key_at = [&](int e) -> uint64_t {
        const int ec = e < n ? e : 0;
        const int sl = slot[ec];
        const uint64_t r = static_cast<uint64_t>(__double_as_longlong(res[ec]));
        return (e < n && sl >= 0) ? r : kInfKey;
    };
    KeyStat ks{~0ull, 0ull, 0, 0};
    uint64_t nan_min = ~0ull;
    for (int rd = 0; rd < 2; ++rd) {
        uint64_t key[RT];
#pragma unroll
        for (int q = 0; q < RT; ++q) key[q] = key_at((rd * RT + q) * NT + tid);
#pragma unroll
        for (int q = 0; q < RT; ++q) {
            if (key[q] < kInfKey) { ks.mn = key[q] < ks.mn ? key[q] : ks.mn; ks.mx = key[q] > ks.mx ? key[q] : ks.mx; ++ks.cnt; }
            if (key[q] > kInfKey) { ks.nan = 1; nan_min = key[q] < nan_min ? key[q] : nan_min; }
        }
    }
    for (int b = tid; b < NB; b += NT) s_cnt[b] = 0;
    KeyStat tot;
    (void)block_excl_scan_dpp<NT>(ks, KeyStat{~0ull, 0ull, 0, 0}, keystat_op, s_ks, &tot);
    const int cnt = tot.cnt;
    if (cnt == 0) return;                                    // too few correspondences: the PKO launch reports it
    if (tot.nan) {                                           // as exact_scale_c_body: the smallest NaN key's thread
        if (nan_min != ~0ull) st->scale = sqrt(__longlong_as_double(static_cast<long long>(nan_min))) / 6.0;
        return;
    }
    const uint64_t range = tot.mx - tot.mn;
    const int bl = range ? 64 - __clzll(static_cast<long long>(range)) : 0;
    int lb = 0;
    while ((1 << (lb + 1)) <= NB) ++lb;
    const int shift = bl > lb ? bl - lb : 0;
    auto bin_of = [&](uint64_t k) { return static_cast<int>((k - tot.mn) >> shift); };
    for (int rd = 0; rd < 2; ++rd) {                         // histogram
        uint64_t key[RT];
#pragma unroll
        for (int q = 0; q < RT; ++q) key[q] = key_at((rd * RT + q) * NT + tid);
#pragma unroll
        for (int q = 0; q < RT; ++q) if (key[q] < kInfKey) atomicAdd(&s_cnt[bin_of(key[q])], 1);
    }
    __syncthreads();
    constexpr int BPT = NB / NT > 0 ? NB / NT : 1;
    int bsum = 0;
    for (int i = 0; i < BPT; ++i) bsum += tid * BPT + i < NB ? s_cnt[tid * BPT + i] : 0;
    int bex = block_excl_scan_dpp<NT>(bsum, 0, [](int a, int c) { return a + c; }, S.wi);
    for (int i = 0; i < BPT; ++i) if (tid * BPT + i < NB) { s_end[tid * BPT + i] = bex; bex += s_cnt[tid * BPT + i]; }
    __syncthreads();
    for (int rd = 0; rd < 2; ++rd) {                         // scatter into bin order
        uint64_t key[RT];
#pragma unroll
        for (int q = 0; q < RT; ++q) key[q] = key_at((rd * RT + q) * NT + tid);
#pragma unroll
        for (int q = 0; q < RT; ++q) if (key[q] < kInfKey) s_tmp[atomicAdd(&s_end[bin_of(key[q])], 1)] = key[q];
    }
    __syncthreads();
    uint64_t kk[2 * RT];                                     // each key's rank in its bin, then the moves
    int pos[2 * RT];
#pragma unroll
    for (int i = 0; i < 2 * RT; ++i) {
        const int p = tid + i * NT;
        pos[i] = -1;
        kk[i] = 0;
        if (p < cnt) {
            const uint64_t k = s_tmp[p];
            const int b = bin_of(k), e = s_end[b], s0 = e - s_cnt[b];
            int r = 0;
            for (int q = s0; q < e; ++q) {
                const uint64_t o = s_tmp[q];
                r += (o < k || (o == k && q < p)) ? 1 : 0;
            }
            kk[i] = k;
            pos[i] = s0 + r;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2 * RT; ++i) if (pos[i] >= 0) s_tmp[pos[i]] = kk[i];
    __syncthreads();
    double* s_x = reinterpret_cast<double*>(s_tmp);          // non-negative keys are their doubles' bits
    const double sum = chain_sum_tx<NT>(s_x, cnt, S);        // std::accumulate, one rounding per add
    const double mean = sum / cnt;
    for (int p = tid; p < cnt; p += NT) { const double v = s_x[p]; s_x[p] = (v - mean) * (v - mean); }
    __syncthreads();
    double var = chain_sum_tx<NT>(s_x, cnt, S);
    var /= cnt;
    if (tid == 0) st->scale = sqrt(var) / 6.0;               // :313-315
}
// A scan counted on the device (lo_icp_optimize_raw: the voxel filter's output count stays in HBM; the host knows only
// the bound ceil(n_raw / stride)): the width is chosen from the count itself, so a 14k-point bound whose filtered scan
// holds 4k points runs the 4k-point sort and sums.  Dynamic LDS: kScaleWideLds (every width fits in it).
__global__ __launch_bounds__(kScaleC) void k_exact_scale_cd(KParams P) {
    if (P.st->done) return;
    extern __shared__ uint64_t s_dyn[];
    __shared__ MonoScratch<kScaleC> S;
    __shared__ KeyStat s_ks[kScaleC / kWave];
    const int n = min(scan_n(P), P.n);                       // the count never exceeds the bound the grid was sized for
    if (n <= kScaleC) exact_scale_c_body<1>(P, n, s_dyn, S, s_ks);
    else if (n <= 2 * kScaleC) exact_scale_c_body<2>(P, n, s_dyn, S, s_ks);
    else if (n <= 3 * kScaleC) exact_scale_c_body<3>(P, n, s_dyn, S, s_ks);
    else if (n <= 4 * kScaleC) exact_scale_c_body<4>(P, n, s_dyn, S, s_ks);
    else if (n <= 5 * kScaleC) exact_scale_c_body<5>(P, n, s_dyn, S, s_ks);
    else if (n <= 6 * kScaleC) exact_scale_c_body<6>(P, n, s_dyn, S, s_ks);
    else if (n <= 8 * kScaleC) exact_scale_c_body<8>(P, n, s_dyn, S, s_ks);
    else exact_scale_c_wide(P, n, s_dyn, S, s_ks);
}
// batched (lo_batch_* over reference-exact contexts): one workgroup per job
template <int PT>
__global__ __launch_bounds__(kScaleC) void k_exact_scale_cb(const KParams* __restrict__ PB) {
    const KParams& P = PB[blockIdx.x];
    if (P.st->done) return;
    extern __shared__ uint64_t s_dyn[];
    __shared__ MonoScratch<kScaleC> S;
    __shared__ KeyStat s_ks[kScaleC / kWave];
    exact_scale_c_body<PT>(P, scan_n(P), s_dyn, S, s_ks);
}
template <int PT>
static hipError_t scale_c_attr() {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_exact_scale_cb<PT>), hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(scale_c_lds<PT>()));
    return hipFuncSetAttribute(reinterpret_cast<const void*>(k_exact_scale_c<PT>), hipFuncAttributeMaxDynamicSharedMemorySize,
                               static_cast<int>(scale_c_lds<PT>()));
}
hipError_t exact_scale_c_prepare() {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_exact_scale_cd), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       static_cast<int>(std::max(kScaleWideLds, scale_c_lds<8>())));
    for (hipError_t r : {scale_c_attr<1>(), scale_c_attr<2>(), scale_c_attr<3>(), scale_c_attr<4>(), scale_c_attr<5>(),
                         scale_c_attr<6>(), scale_c_attr<8>(), scale_c_attr<16>()})
        if (e == hipSuccess) e = r;
    return e;
}
// jobs [0, njobs) of PB, every job's P.n <= n_max <= kExactMergeMax
void launch_exact_scale_cb(const KParams* PB, int njobs, int n_max, hipStream_t s) {
    const dim3 g(njobs), b(kScaleC);
    if (n_max <= kScaleC) hipLaunchKernelGGL(k_exact_scale_cb<1>, g, b, scale_c_lds<1>(), s, PB);
    else if (n_max <= 2 * kScaleC) hipLaunchKernelGGL(k_exact_scale_cb<2>, g, b, scale_c_lds<2>(), s, PB);
    else if (n_max <= 3 * kScaleC) hipLaunchKernelGGL(k_exact_scale_cb<3>, g, b, scale_c_lds<3>(), s, PB);
    else if (n_max <= 4 * kScaleC) hipLaunchKernelGGL(k_exact_scale_cb<4>, g, b, scale_c_lds<4>(), s, PB);
    else if (n_max <= 5 * kScaleC) hipLaunchKernelGGL(k_exact_scale_cb<5>, g, b, scale_c_lds<5>(), s, PB);
    else if (n_max <= 6 * kScaleC) hipLaunchKernelGGL(k_exact_scale_cb<6>, g, b, scale_c_lds<6>(), s, PB);
    else hipLaunchKernelGGL(k_exact_scale_cb<8>, g, b, scale_c_lds<8>(), s, PB);
}
// P.n <= kExactScaleCMax; a device-counted scan (P.n_dev) chooses its width from the count on the device
void launch_exact_scale_c(const KParams& P, hipStream_t s) {
    if (P.n_dev && P.n > kScaleC) {
        const size_t lds = P.n > 8 * kScaleC ? std::max(kScaleWideLds, scale_c_lds<8>()) : scale_c_lds<8>();
        hipLaunchKernelGGL(k_exact_scale_cd, dim3(1), dim3(kScaleC), lds, s, P);
    } else if (P.n <= kScaleC) hipLaunchKernelGGL(k_exact_scale_c<1>, dim3(1), dim3(kScaleC), scale_c_lds<1>(), s, P);
    else if (P.n <= 2 * kScaleC) hipLaunchKernelGGL(k_exact_scale_c<2>, dim3(1), dim3(kScaleC), scale_c_lds<2>(), s, P);
    // keys per thread = ceil(n / 1024) up to 6 (the kernel's time grows with the width: KITTI scans of 4-5k points
    // took the 8-wide sort at 33 us against 22 us for the 4-wide one)
    else if (P.n <= 3 * kScaleC) hipLaunchKernelGGL(k_exact_scale_c<3>, dim3(1), dim3(kScaleC), scale_c_lds<3>(), s, P);
    else if (P.n <= 4 * kScaleC) hipLaunchKernelGGL(k_exact_scale_c<4>, dim3(1), dim3(kScaleC), scale_c_lds<4>(), s, P);
    else if (P.n <= 5 * kScaleC) hipLaunchKernelGGL(k_exact_scale_c<5>, dim3(1), dim3(kScaleC), scale_c_lds<5>(), s, P);
    else if (P.n <= 6 * kScaleC) hipLaunchKernelGGL(k_exact_scale_c<6>, dim3(1), dim3(kScaleC), scale_c_lds<6>(), s, P);
    else if (P.n <= 8 * kScaleC) hipLaunchKernelGGL(k_exact_scale_c<8>, dim3(1), dim3(kScaleC), scale_c_lds<8>(), s, P);
    else hipLaunchKernelGGL(k_exact_scale_c<16>, dim3(1), dim3(kScaleC), scale_c_lds<16>(), s, P);
}

constexpr int kScaleThreads = 256;                           // k_exact_scale_s: 4 waves, PT = padded size / 256
template <int PT>
static hipError_t scale_s_attr() {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(k_exact_scale_s<kScaleThreads, PT>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(PT * kScaleThreads * sizeof(double)));
}
// The kernels' dynamic LDS (up to 64 KB), set on the calling thread's current device (exact_prepare, per context).
hipError_t exact_scale_m_prepare() {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_rank_runs), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       static_cast<int>(kExactMergeMax * sizeof(uint64_t)));
    for (hipError_t r : {scale_s_attr<1>(), scale_s_attr<2>(), scale_s_attr<4>(), scale_s_attr<8>(), scale_s_attr<16>(),
                         scale_s_attr<32>()})
        if (e == hipSuccess) e = r;
    return e;
}
// P.nb runs of 256 sorted keys (P.nb * 256 <= kExactMergeMax) -> sorted (P.nb * 256 keys of scratch) -> the scale
void launch_exact_scale_m(const KParams& P, const uint64_t* runs, uint64_t* sorted, hipStream_t s) {
    const int need = P.nb * kBlock;
    hipLaunchKernelGGL(k_rank_runs, dim3(P.nb), dim3(kBlock), static_cast<size_t>(need) * sizeof(uint64_t), s, P, runs, sorted);
    const size_t lds = kScaleThreads * sizeof(double);
    constexpr int T = kScaleThreads;
    if (need <= T) hipLaunchKernelGGL((k_exact_scale_s<T, 1>), dim3(1), dim3(T), lds, s, P, sorted);
    else if (need <= 2 * T) hipLaunchKernelGGL((k_exact_scale_s<T, 2>), dim3(1), dim3(T), 2 * lds, s, P, sorted);
    else if (need <= 4 * T) hipLaunchKernelGGL((k_exact_scale_s<T, 4>), dim3(1), dim3(T), 4 * lds, s, P, sorted);
    else if (need <= 8 * T) hipLaunchKernelGGL((k_exact_scale_s<T, 8>), dim3(1), dim3(T), 8 * lds, s, P, sorted);
    else if (need <= 16 * T) hipLaunchKernelGGL((k_exact_scale_s<T, 16>), dim3(1), dim3(T), 16 * lds, s, P, sorted);
    else hipLaunchKernelGGL((k_exact_scale_s<T, 32>), dim3(1), dim3(T), 32 * lds, s, P, sorted);
}

// ---- iteration 0 for scans beyond the one-workgroup sort (kExactMaxPoints < n): k_exact_resid writes every point's
// residual (+inf without a correspondence) to global memory, the context sorts them ascending (hipCUB radix sort:
// the same order as std::sort for the non-NaN values; -0 / +0 ties do not change any sum), and launch_mwm_scale runs
// both sequential sums over the sorted residuals across the chip (lo_seqsum.h MwmBuf, kernels k_mwm_* below) ----
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
static hipError_t scale_attr() {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(k_exact_scale<PT>), hipFuncAttributeMaxDynamicSharedMemorySize,
                               kSeqThreads * PT * 8);
}
// k_exact_scale's dynamic LDS (up to 128 KB), set on the calling thread's current device (exact_prepare, per context)
hipError_t exact_scale_rank_prepare() {
    hipError_t e = hipSuccess;
    for (hipError_t r : {scale_attr<1>(), scale_attr<2>(), scale_attr<3>(), scale_attr<4>(), scale_attr<5>(), scale_attr<6>(),
                         scale_attr<7>(), scale_attr<8>(), scale_attr<10>(), scale_attr<12>(), scale_attr<16>()})
        if (e == hipSuccess) e = r;
    return e;
}
template <int PT>
static void launch_scale_pt(const KParams& P, const double* sorted, hipStream_t s) {
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
    // row-major [point][43], or term-major [43][ex_ld] (coalesced columns for the column sums, launch_mw_sums)
    const size_t o0 = P.ex_ld ? static_cast<size_t>(i) : static_cast<size_t>(i) * kExactTerms;
    const size_t os = P.ex_ld ? static_cast<size_t>(P.ex_ld) : 1;
    float* out = P.ex_terms + o0;
    const int s = P.slot[i];
    // term-major (long sums): the point's 14 factor rows only -- the readers form each term as the same fp32 product
    // (launch_mw_sums factored); row-major: the 43 products
    const int nout = P.ex_ld && kExactFactored ? kExactFactors : kExactTerms;
    if (s < 0) {
        for (int k = 0; k < nout; ++k) out[k * os] = 0.0f;
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
    if (P.ex_ld && kExactFactored) {
#pragma unroll
        for (int k = 0; k < kExactFactors; ++k) out[k * os] = f[k];
        return;
    }
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

// ---- long columns across the chip (lo_seqsum.h "Long signed fp32 columns"): chunk sums -> classification -> walk ----
// The edge margin M = 2^(E - kMwEdgeBits) of a predicted binade E (lo_seqsum.h): a term whose predicted prefix lies
// closer to an edge heads a segment, and a segment's check allows a deviation of M minus its length's half-ulps.  A
// narrower margin trades heads for failed checks (segments summed term by term); same-box A/B on the C5 scans
// (`make edge`, scripts/gpu_r05_edge.sh): 9 / 10 / 11 bits -> 434 / 462 / 448 scans/s, heads per scan 355k / 225k /
// 145k, chunks run term by term 78 / 47 / 44, failed segments 950 / 1447 / 2301 (bitwise the same).
#ifndef LO_MW_EDGE_BITS
#define LO_MW_EDGE_BITS 10
#endif
constexpr int kMwEdgeBits = LO_MW_EDGE_BITS;
#ifndef LO_MW_REG_HEADS
#define LO_MW_REG_HEADS 2
#endif
constexpr int kMwRegHeads = LO_MW_REG_HEADS;                  // classification: heads per thread kept in registers
constexpr int kMwChainAgain = 1;                              // the walk: failures per window followed by a chain
static_assert(kMwEdgeBits >= 1 && kMwEdgeBits <= 11, "a 4096-term segment must fit the margin: 2^(23 - bits) > 2049");
__device__ __forceinline__ int mw_n(int n_cap, const int* n_dev) { return n_dev ? *n_dev : n_cap; }
// Column colI of the long sums, from term off on: a stored column (col0 + colI * ld), or (FAC) the fp32 product of
// its two factor rows (exact_term_factors: the 43 terms are products of a point's 14 factors, so k_exact_terms writes
// 14 rows instead of 43 columns and every reader forms the same product)
template <bool FAC> struct MwCol {
    const float* a;
    const float* b;
    __device__ __forceinline__ MwCol(const float* col0, int ld, int colI, int off) {
        if constexpr (FAC) {
            int fa, fb;
            exact_term_factors(colI, fa, fb);
            a = col0 + static_cast<size_t>(fa) * ld + off;
            b = col0 + static_cast<size_t>(fb) * ld + off;
        } else {
            a = col0 + static_cast<size_t>(colI) * ld + off;
            b = nullptr;
        }
    }
    __device__ __forceinline__ float operator[](int j) const {
        if constexpr (FAC) return a[j] * b[j];
        else return a[j];
    }
    // terms base .. base + kMwPT - 1 (0 from lim on): 16-B loads when the run is whole and aligned (a thread's 16
    // consecutive terms as 4 dwordx4 loads per row instead of 16 dword loads, each touching 64 lanes' lines)
    __device__ __forceinline__ void load_run(int base, int lim, float (&v)[kMwPT]) const {
        static_assert(kMwPT % 4 == 0, "whole float4s");
        uintptr_t al = reinterpret_cast<uintptr_t>(a + base);
        if constexpr (FAC) al |= reinterpret_cast<uintptr_t>(b + base);
        if (base + kMwPT <= lim && (al & 15) == 0) {
            const float4* pa = reinterpret_cast<const float4*>(a + base);
#pragma unroll
            for (int q = 0; q < kMwPT / 4; ++q) {
                const float4 x = pa[q];
                v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
            }
            if constexpr (FAC) {
                const float4* pb = reinterpret_cast<const float4*>(b + base);
#pragma unroll
                for (int q = 0; q < kMwPT / 4; ++q) {
                    const float4 y = pb[q];
                    v[4 * q] *= y.x; v[4 * q + 1] *= y.y; v[4 * q + 2] *= y.z; v[4 * q + 3] *= y.w;
                }
            }
        } else {
#pragma unroll
            for (int q = 0; q < kMwPT; ++q) v[q] = base + q < lim ? (*this)[base + q] : 0.0f;
        }
    }
};

template <bool FAC>
__global__ __launch_bounds__(256) void k_mw_chunk_sums(const float* __restrict__ col0, int ld, int n_cap,
                                                       const int* n_dev, const DevState* st, MwBuf B) {
    if (st && st->done) return;
    __shared__ double s_w[2][4];
    const int c = blockIdx.x, colI = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int n = mw_n(n_cap, n_dev), c0 = c * kMwChunk, mc = min(kMwChunk, n - c0);
    if (mc <= 0) return;                                       // chunks past the end publish nothing
    const MwCol<FAC> col(col0, ld, colI, c0);
    double v = 0.0, a = 0.0;
#pragma unroll
    for (int k = 0; k < kMwChunk / 256; ++k) {                 // 16 terms per thread, coalesced
        const int j = k * 256 + tid;
        const double x = j < mc ? static_cast<double>(col[j]) : 0.0;
        v += x;
        a += fabs(x);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { v += __shfl_xor(v, o, 64); a += __shfl_xor(a, o, 64); }
    if (lane == 0) { s_w[0][wid] = v; s_w[1][wid] = a; }
    __syncthreads();
    if (tid == 0) {
        const size_t o = static_cast<size_t>(colI) * B.nchunks + c;
        B.csum[o] = ((s_w[0][0] + s_w[0][1]) + s_w[0][2]) + s_w[0][3];
        B.cabs[o] = ((s_w[1][0] + s_w[1][1]) + s_w[1][2]) + s_w[1][3];
    }
}

constexpr int kMwWaves = kMwThreads / kWave;
struct MwScratch {
    double wd[kMwWaves];
    double wd2[2 * kMwWaves];
    long long wl[kMwWaves];
    int wi[kMwWaves];
    int elast[kMwThreads];
    int glast[kMwThreads];
    int h_idx[kMwCap];
    int h_e[kMwCap];
    long long h_p[kMwCap];
    double h_t[kMwCap];
};

// The chunk's prediction base: the chunk sums (+ modelled drift, DRIFT) of the chunks before it, and the magnitude sum
// through this chunk.  Every thread returns both.
template <bool DRIFT>
__device__ __forceinline__ void mw_base(const MwBuf& B, size_t co, int c, double* s_w, double& T0, double& A) {
    double t0 = 0.0, a0 = 0.0;
    for (int k = threadIdx.x; k <= c; k += kMwThreads) {
        if (k < c) t0 += DRIFT ? B.csum[co + k] + B.dcorr[co + k] : B.csum[co + k];
        a0 += B.cabs[co + k];
    }
    (void)block_excl_scan<double, kMwThreads>(t0, s_w, T0);
    (void)block_excl_scan<double, kMwThreads>(a0, s_w, A);
}

// One thread's share of a chunk's modelled drift: each step's rounding in its predicted binade (tex: the predicted sum
// before the thread's first term).
__device__ __forceinline__ double mw_drift_terms(const float (&v)[kMwPT], double tex) {
    double d = 0.0, tl = 0.0;
#pragma unroll
    for (int a = 0; a < kMwPT; ++a) {
        tl += static_cast<double>(v[a]);
        const int E = binade_abs(tex + tl);
        const double x = static_cast<double>(v[a]);
        const double q = ldexp(rint(ldexp(x, 23 - E)), E - 23) - x;   // branch-free: no binade -> not counted
        d += E != kExpNone ? q : 0.0;
    }
    return d;
}

template <bool FAC>
__global__ __launch_bounds__(kMwThreads) void k_mw_drift(const float* __restrict__ col0, int ld, int n_cap,
                                                        const int* n_dev, const DevState* st, MwBuf B) {
    if (st && st->done) return;
    __shared__ double s_w[kMwWaves];
    const int c = blockIdx.x, colI = blockIdx.y, tid = threadIdx.x;
    const int n = mw_n(n_cap, n_dev), c0 = c * kMwChunk, mc = min(kMwChunk, n - c0);
    const size_t co = static_cast<size_t>(colI) * B.nchunks;
    if (mc <= 0) return;
    const MwCol<FAC> col(col0, ld, colI, c0);
    double T0, A;
    mw_base<false>(B, co, c, s_w, T0, A);
    const int base = tid * kMwPT;
    float v[kMwPT];
    col.load_run(base, mc, v);
    double run = 0.0;
#pragma unroll
    for (int a = 0; a < kMwPT; ++a) run += static_cast<double>(v[a]);
    double ttot;
    const double tex = T0 + block_excl_scan<double, kMwThreads>(run, s_w, ttot);
    double dtot;
    (void)block_excl_scan<double, kMwThreads>(mw_drift_terms(v, tex), s_w, dtot);
    if (tid == 0) B.dcorr[co + c] = dtot;
}

// Chunk values handed from one classification workgroup to the later chunks of its column inside the launch (the fused
// path below): csum / cabs / dcorr hold kMwUnset until their chunk publishes them with an sc1 store; a reader polls
// with sc1 loads (lo_device.h Mem<true>).  k_mw_compact puts kMwUnset back after the launch, mw_clear sets it at
// allocation.  Computed values are never kMwUnset (a NaN is published as the canonical quiet NaN).  A wait is bounded
// by kMwWaitTicks of the 100 MHz clock and then reads 0: any prediction is correct (the walk checks every head), a
// wrong one only costs term-by-term segments, so no value can hang or corrupt a sum.
constexpr unsigned long long kMwUnset = ~0ull;
constexpr unsigned long long kMwWaitTicks = 10000000ull;      // 0.1 s
__device__ __forceinline__ void mw_publish(double* p, double v) {
    Mem<true>::st(p, v != v ? __builtin_bit_cast(double, 0x7FF8000000000000ull) : v);
}
__device__ __forceinline__ double mw_await(const double* p) {
    unsigned long long b = Mem<true>::ld(reinterpret_cast<const unsigned long long*>(p));
    if (b == kMwUnset) {
        const unsigned long long t0 = wall_clock64();
        do {
            __builtin_amdgcn_s_sleep(1);
            b = Mem<true>::ld(reinterpret_cast<const unsigned long long*>(p));
        } while (b == kMwUnset && wall_clock64() - t0 <= kMwWaitTicks);
    }
    return b == kMwUnset ? 0.0 : __builtin_bit_cast(double, b);
}
// Two sums over the workgroup (every thread gets both; s_w: 2 * kMwWaves entries, free again on return).
__device__ __forceinline__ void mw_block_sum2(double& x, double& y, double* s_w) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { x += __shfl_xor(x, o, 64); y += __shfl_xor(y, o, 64); }
    if (lane == 0) { s_w[wid] = x; s_w[kMwWaves + wid] = y; }
    __syncthreads();
    x = 0.0;
    y = 0.0;
#pragma unroll
    for (int w = 0; w < kMwWaves; ++w) { x += s_w[w]; y += s_w[kMwWaves + w]; }
    __syncthreads();
}

// FUSED (the default): one launch computes each chunk's sums, publishes them, takes the sums of the chunks before it from
// their workgroups (a look-back: every workgroup waits only for lower chunks of its own column, dispatched before it),
// then its modelled drift the same way, then classifies -- k_mw_chunk_sums and k_mw_drift fold in.  The prediction
// base is the same quantity summed in another order (T0 = chunk sums + drift corrections of the chunks before).
// !FUSED: the three-launch path (LO_MW_SPLIT=1, A/B).
template <bool FUSED, bool FAC>
__global__ __launch_bounds__(kMwThreads, 4) void k_mw_classify(const float* __restrict__ col0, int ld, int n_cap,
                                                             const int* n_dev, const DevState* st, MwBuf B) {
    if (st && st->done) return;
    __shared__ MwScratch S;
    const int c = blockIdx.x, colI = blockIdx.y, tid = threadIdx.x;
    const int n = mw_n(n_cap, n_dev), c0 = c * kMwChunk, mc = min(kMwChunk, n - c0);
    const size_t co = static_cast<size_t>(colI) * B.nchunks;
    if (mc <= 0) {
        if (tid == 0) B.nh[co + c] = 0;
        return;
    }
    const MwCol<FAC> col(col0, ld, colI, c0);
    const int base = tid * kMwPT;
    float v[kMwPT];
    col.load_run(base, mc, v);
    double run = 0.0;
#pragma unroll
    for (int a = 0; a < kMwPT; ++a) run += static_cast<double>(v[a]);
    double T0, A, ttot, ex;
    if constexpr (FUSED) {
        ex = block_excl_scan<double, kMwThreads>(run, S.wd, ttot);
        double ab = 0.0, unused = 0.0;
#pragma unroll
        for (int a = 0; a < kMwPT; ++a) ab += fabs(static_cast<double>(v[a]));
        mw_block_sum2(ab, unused, S.wd2);
        if (tid == 0) { mw_publish(B.csum + co + c, ttot); mw_publish(B.cabs + co + c, ab); }
        double t0 = 0.0, a0 = 0.0;
        for (int k = tid; k < c; k += kMwThreads) { t0 += mw_await(B.csum + co + k); a0 += mw_await(B.cabs + co + k); }
        mw_block_sum2(t0, a0, S.wd2);
        A = a0 + ab;
        double d = mw_drift_terms(v, t0 + ex), dp = 0.0;
        mw_block_sum2(d, dp, S.wd2);
        if (tid == 0) mw_publish(B.dcorr + co + c, d);
        for (int k = tid; k < c; k += kMwThreads) dp += mw_await(B.dcorr + co + k);
        double unused2 = 0.0;
        mw_block_sum2(dp, unused2, S.wd2);
        T0 = t0 + dp;
    } else {
        mw_base<true>(B, co, c, S.wd, T0, A);
        ex = block_excl_scan<double, kMwThreads>(run, S.wd, ttot);
    }
    const double eps_t = ldexp(A + fabs(T0), -45);             // bound on the in-chunk prediction error (see above)
    const double tex = T0 + ex;
    {
        const double Tl = tex + run;
        S.elast[tid] = binade_abs(Tl);
        S.glast[tid] = static_cast<int>(__builtin_bit_cast(uint64_t, Tl) >> 63);
    }
    __syncthreads();
    const int e_in = tid ? S.elast[tid - 1] : kExpNone, g_in = tid ? S.glast[tid - 1] : 0;
    // heads: binade / sign changes, edge proximity, halfway ties; term 0 of every chunk heads a segment
    auto classify = [&](int a, double T, int ep, int gp, int& E, int& G, long long& qa) -> bool {
        const int j = base + a;
        const float xv = v[a];
        // branch-free, on T's bits.  G: the sign bit (it matters only where E and the previous E are binades -- else
        // the term heads anyway -- and there it is the sign).  Edge proximity: |T| = 2^E (1 + m) lies within
        // M = 2^(E - kMwEdgeBits) of an edge <=> m's top kMwEdgeBits bits are all zero, or all one with a nonzero rest
        // (kMwEdgeBits <= 11: the top bits sit in the high word)
        const uint64_t tb = __builtin_bit_cast(uint64_t, T);
        const uint32_t hi = static_cast<uint32_t>(tb >> 32), lo32 = static_cast<uint32_t>(tb);
        E = binade_abs(T);
        G = static_cast<int>(hi >> 31);
        const uint32_t top = (hi >> (20 - kMwEdgeBits)) & ((1u << kMwEdgeBits) - 1);
        const bool rest = ((hi & ((1u << (20 - kMwEdgeBits)) - 1)) | lo32) != 0;
        const bool edge = E == kExpNone || top == 0 || (top == (1u << kMwEdgeBits) - 1 && rest);
        const double t = ldexp(static_cast<double>(xv), 23 - E);   // |t| < 2^24 whenever the term does not head
        const double r = rint(t);
        const bool live = j < mc && (xv != 0.0f || j == 0);
        const bool head = live && (edge || E != ep || G != gp || j == 0 || fabs(t - r) == 0.5);   // |t - r| = 1/2: a tie
        qa = static_cast<long long>(static_cast<int>(live && !head ? r : 0.0));
        return head;
    };
    long long ql = 0;
    int nhl = 0;
    // the first kMwRegHeads heads of the thread kept in registers: when no thread of the workgroup has more, the
    // record pass below is skipped (same-box A/B, C5 exact scans/s: 0 / 1 / 2 / 3 heads -> 558 / 584 / 585 / 581;
    // keeping them also ends the kernel's scratch spill)
    int r_a[kMwRegHeads + 1], r_e[kMwRegHeads + 1], r_q[kMwRegHeads + 1];
    double r_t[kMwRegHeads + 1];
    {
        double tl = 0.0;
        int ep = e_in, gp = g_in;
#pragma unroll
        for (int a = 0; a < kMwPT; ++a) {
            tl += static_cast<double>(v[a]);
            const double T = tex + tl;
            int E, G;
            long long qa;
            const bool hd = classify(a, T, ep, gp, E, G, qa);
#pragma unroll
            for (int r = 0; r < kMwRegHeads; ++r)
                if (hd && nhl == r) { r_a[r] = a; r_e[r] = E; r_q[r] = static_cast<int>(ql); r_t[r] = T; }
            nhl += hd ? 1 : 0;
            ql += qa;
            ep = E;
            gp = G;
        }
    }
    // the record pass below recomputes every term's classification: opaque copies of the terms keep the compiler from
    // carrying the first pass's per-term values across the scans (190 -> fewer VGPRs, more waves per SIMD)
#pragma unroll
    for (int a = 0; a < kMwPT; ++a) asm volatile("" : "+v"(v[a]));
    long long ptot;
    const long long pex = block_excl_scan<long long, kMwThreads>(ql, S.wl, ptot);
    int htot;
    const int hbase = block_excl_scan<int, kMwThreads>(nhl, S.wi, htot);
    const size_t rb = (co + c) * kMwCap;
    if (htot > kMwCap) {                                       // uniform: the whole chunk as one term-by-term run
        if (tid == 0) {
            B.nh[co + c] = 1;
            B.idx[rb] = c0;
            B.end[rb] = c0 + mc;
            B.x[rb] = col[0];
            B.dq[rb] = -0.0f;
            B.flag[rb] = kMwFail;
            B.dlo[rb] = __builtin_inf();
            B.dhi[rb] = -__builtin_inf();
        }
        return;
    }
    if (kMwRegHeads > 0 && !__syncthreads_or(nhl > kMwRegHeads)) {   // uniform
#pragma unroll
        for (int r = 0; r < kMwRegHeads; ++r)
            if (r < nhl) { S.h_idx[hbase + r] = base + r_a[r]; S.h_e[hbase + r] = r_e[r]; S.h_p[hbase + r] = pex + r_q[r]; S.h_t[hbase + r] = r_t[r]; }
    } else {
        double tl = 0.0;
        int ep = e_in, gp = g_in, hk = hbase;
        long long prun = pex;
#pragma unroll
        for (int a = 0; a < kMwPT; ++a) {
            tl += static_cast<double>(v[a]);
            const double T = tex + tl;
            int E, G;
            long long qa;
            const bool hd = classify(a, T, ep, gp, E, G, qa);
            prun += qa;
            if (hd) { S.h_idx[hk] = base + a; S.h_e[hk] = E; S.h_p[hk] = prun; S.h_t[hk] = T; ++hk; }
            ep = E;
            gp = G;
        }
    }
    __syncthreads();
    for (int k = tid; k < htot; k += kMwThreads) {             // one record per head
        const int hi = S.h_idx[k], E = S.h_e[k];
        const long long hp = S.h_p[k];
        const double ht = S.h_t[k];
        const bool last = k + 1 >= htot;
        const int hend = last ? mc : S.h_idx[k + 1];
        const long long pend = last ? ptot : S.h_p[k + 1];
        int flag = hend > hi + 1 ? 0 : 1;
        double dlo = __builtin_inf(), dhi = -__builtin_inf();
        float dq = -0.0f;
        if (!flag) {
            flag = kMwFail;
            if (E != kExpNone) {
                const double u = ldexp(1.0, E - 23), lo = ldexp(1.0, E);
                const double dev = ldexp(1.0, E - kMwEdgeBits) - (static_cast<double>(hend - hi) * 0.5 + 1.0) * u - 2.0 * eps_t;
                if (dev >= 0.0) {
                    // |d - ht| <= dev, rounded inwards; the binade of the head's sign, its top end exclusive
                    const double slack = ldexp(fabs(ht) + dev, -51);
                    const double top = 2.0 * lo - ldexp(lo, -52);
                    dlo = (ht - dev) + slack;
                    dhi = (ht + dev) - slack;
                    if (ht > 0.0) { dlo = fmax(dlo, lo); dhi = fmin(dhi, top); }
                    else { dlo = fmax(dlo, -top); dhi = fmin(dhi, -lo); }
                    dq = static_cast<float>(static_cast<double>(pend - hp) * u);
                    flag = 0;
                }
            }
        }
        const size_t r = rb + k;
        B.idx[r] = c0 + hi;
        B.end[r] = c0 + hend;
        B.x[r] = col[hi];
        B.dq[r] = dq;
        B.flag[r] = flag;
        B.dlo[r] = dlo;
        B.dhi[r] = dhi;
    }
    if (tid == 0) B.nh[co + c] = htot;
}

// s + col[j0] + ... + col[j1 - 1] term by term (one wave, wave-uniform).  The terms come in through scalar loads, 32 at a
// time with the next 32 in flight, so the chain is one v_add_f32 per term with an SGPR operand (no readlane hazards).
template <bool FAC>
__device__ __forceinline__ float walk_terms(const MwCol<FAC>& col, int j0, int j1, float s) {
    constexpr int kB = 32;
    j0 = __builtin_amdgcn_readfirstlane(j0);
    j1 = __builtin_amdgcn_readfirstlane(j1);
    const int lane = threadIdx.x & 63;
    int j = j0;
    {                                                          // to a 128-byte boundary: one load per lane
        const int a = min(j1, (j0 + kB - 1) & ~(kB - 1));
        const float v = lane < a - j0 ? col[j0 + lane] : -0.0f;
        for (int l = 0; l < a - j0; ++l) s = s + __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
        j = a;
    }
    if (j + kB <= j1) {
        float cur[kB], nxt[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) cur[u] = col[j + u];
        for (; j + 2 * kB <= j1; j += kB) {
#pragma unroll
            for (int u = 0; u < kB; ++u) nxt[u] = col[j + kB + u];
#pragma unroll
            for (int u = 0; u < kB; ++u) s = s + cur[u];
#pragma unroll
            for (int u = 0; u < kB; ++u) cur[u] = nxt[u];
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) s = s + cur[u];
        j += kB;
    }
    {                                                          // the rest (< kB terms): one load per lane
        const float v = lane < j1 - j ? col[j + lane] : -0.0f;
        for (int l = 0; l < j1 - j; ++l) s = s + __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
    }
    // every load above complete (vmcnt(0)): a caller's loop then carries no possibly-pending register, which would make
    // the compiler wait for ALL loads at the loop head -- the walk's next-window prefetch included
    __builtin_amdgcn_s_waitcnt(0x0F70);
    return s;
}

// Compaction: chunk c's records to their place in the column's walk order (offset = the heads of the chunks before it).
__global__ __launch_bounds__(256) void k_mw_compact(int n_cap, const int* n_dev, const DevState* st, MwBuf B) {
    if (st && st->done) return;
    __shared__ int s_w[4];
    const int c = blockIdx.x, colI = blockIdx.y, tid = threadIdx.x;
    const int n = mw_n(n_cap, n_dev), nc = (n + kMwChunk - 1) / kMwChunk;
    if (c >= nc) return;
    const size_t co = static_cast<size_t>(colI) * B.nchunks;
    int before = 0;
    for (int k = tid; k < c; k += 256) before += B.nh[co + k];
    int off;
    (void)block_excl_scan<int, 256>(before, s_w, off);
    const int h = B.nh[co + c];
    if (tid == 0) {                                            // the chunk's handed-off values back to unset
        const double u = __builtin_bit_cast(double, kMwUnset);
        B.csum[co + c] = u;
        B.cabs[co + c] = u;
        B.dcorr[co + c] = u;
    }
    const size_t src = (co + c) * kMwCap, dst = static_cast<size_t>(colI) * B.cstride + off;
    for (int k = tid; k < h; k += 256) {
        B.c_idx[dst + k] = B.idx[src + k];
        B.c_end[dst + k] = B.end[src + k];
        B.c_x[dst + k] = B.x[src + k];
        B.c_dq[dst + k] = B.dq[src + k];
        B.c_flag[dst + k] = B.flag[src + k];
        B.c_dlo[dst + k] = B.dlo[src + k];
        B.c_dhi[dst + k] = B.dhi[src + k];
    }
    if (c == nc - 1) {                                         // no-op records after the last head
        if (tid < kMwPad) {
            const size_t r = dst + h + tid;
            B.c_idx[r] = 0; B.c_end[r] = 0; B.c_flag[r] = 1; B.c_x[r] = -0.0f; B.c_dq[r] = -0.0f;
            B.c_dlo[r] = 0.0; B.c_dhi[r] = 0.0;
        }
        if (tid == 0) B.ntot[colI] = off + h;
    }
}

// One wave per column: every head in order, a window of 64 heads at a time (the next window's records in flight).
// The fast path adds the window's heads as a plain fp32 chain -- s += x (the head's own step), s += dq (its segment)
// -- storing the sum right after head l's step to LDS (lane l reads it back); the 64 checks then run lane-parallel.  A
// failed check at head f restarts from its recorded sum (exact: every earlier head passed), sums f's segment term by
// term and chains the window's later heads again.  stats (nullable, per column): heads, segments summed term by term, chunks that were one
// term-by-term run.
template <bool FAC>
__global__ __launch_bounds__(64) void k_mw_walk(const float* __restrict__ col0, int ld, int n_cap, const int* n_dev,
                                                const DevState* st, MwBuf B, float* out, long long* stats) {
    if (st && st->done) return;
    const int lane = threadIdx.x, colI = blockIdx.x;
    const int n = mw_n(n_cap, n_dev);
    const MwCol<FAC> col(col0, ld, colI, 0);
    const size_t rb = static_cast<size_t>(colI) * B.cstride;
    const int total = n > 0 ? B.ntot[colI] : 0;
    struct Win { int hi, end, flag; float x, dq; double dlo, dhi; };
    auto load = [&](int k0) {                                  // records past the last head are no-ops (kMwPad)
        const size_t r = rb + k0 + lane;
        return Win{B.c_idx[r], B.c_end[r], B.c_flag[r], B.c_x[r], B.c_dq[r], B.c_dlo[r], B.c_dhi[r]};
    };
    auto rlf = [](float v, int l) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l)); };
    float s = 0.0f;
    int fbs = 0, chained = 0;
#ifdef LO_EXACT_STAMPS
    // cycle split: chained chunks / failed segments (walk_terms) / the slow paths in all, and the whole walk
    unsigned long long t_ch = 0, t_fs = 0, t_slow = 0;
    const unsigned long long t_begin = __builtin_amdgcn_s_memtime();
#define LO_WALK_TERMS(isch, expr) do { const unsigned long long t_w0 = __builtin_amdgcn_s_memtime(); expr; \
        const unsigned long long t_w = __builtin_amdgcn_s_memtime() - t_w0; if (isch) t_ch += t_w; else t_fs += t_w; } while (0)
#else
#define LO_WALK_TERMS(isch, expr) expr
#endif
    // one window: the plain chain, the lane-parallel checks; from a failed check at head f: its segment term by term,
    // then, for the window's first failure, the chain over its later heads only, 8 at a time, and their checks; after
    // that the rest head by head.  Same-box A/B on the C5 scans (scans/s): head by head after any failure 548, the
    // chain again after the first 550, the first two 550, every failure 528 (failures cluster: a poorly predicted
    // stretch fails head after head), a full 64-head chain again after every failure 498
    __shared__ float2 s_xd[64];                                // the window's (x, dq), read back as broadcasts
    __shared__ float s_rec[64 * 64];                           // [head l][lane]: the sum right after head l's step
    auto chain = [&]() -> float {
        __syncthreads();
        float2 xd[64];                                         // every operand in registers before the chain starts:
#pragma unroll                                                 // the chain's LDS stores share the loads' counter
        for (int l = 0; l < 64; ++l) xd[l] = s_xd[l];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int l = 0; l < 64; ++l) {                          // no-op records add -0: s + -0 = s bitwise
            s = s + xd[l].x;
            s_rec[l * 64 + lane] = s;                          // every lane its own word: no bank conflicts
            s = s + xd[l].y;
        }
        __syncthreads();
        return s_rec[lane * 64 + lane];
    };
    // after a failure: the chain over heads [from, m) only, 8 at a time (the window's records below from are no-ops)
    auto chain_from = [&](int from, int m) -> float {
        __syncthreads();
        for (int b = from & ~7; b < m; b += 8) {               // records up to 64 exist (pad: no-ops)
            float2 xd[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) xd[u] = s_xd[b + u];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s = s + xd[u].x;
                s_rec[(b + u) * 64 + lane] = s;
                s = s + xd[u].y;
            }
        }
        __syncthreads();
        return s_rec[lane * 64 + lane];
    };
    auto process = [&](const Win& cur, int k0) {
        s_xd[lane] = make_float2(cur.x, cur.dq);
        float rec = chain();
        const int m = min(64, total - k0);
        int from = 0, nre = 0;                                 // heads below from are summed; nre: chains again
        for (;;) {
            const double d = static_cast<double>(rec);
            const bool ok = lane < from || cur.flag == 1 || (cur.flag == 0 && d >= cur.dlo && d <= cur.dhi);
            const unsigned long long badm = __ballot(!ok);
            if (!badm) return;                                 // uniform
#ifdef LO_EXACT_STAMPS
            const unsigned long long t_s0 = __builtin_amdgcn_s_memtime();
#endif
            const int f = __builtin_ctzll(badm);
            s = rlf(rec, f);                                   // exact: every head before f passed
            const int h = __builtin_amdgcn_readlane(cur.hi, f), end = __builtin_amdgcn_readlane(cur.end, f);
            const bool ch = __builtin_amdgcn_readlane(cur.flag, f) == kMwFail && end - h > 1;
            chained += ch ? 1 : 0;
            LO_WALK_TERMS(ch, s = walk_terms(col, h + 1, end, s));
            ++fbs;
            from = f + 1;
            if (from < m && nre < kMwChainAgain) {                // the chain again over the window's later heads
                ++nre;
                __syncthreads();
                if (lane < from) s_xd[lane] = make_float2(-0.0f, -0.0f);
                rec = chain_from(from, m);
#ifdef LO_EXACT_STAMPS
                t_slow += __builtin_amdgcn_s_memtime() - t_s0;
#endif
                continue;
            }
            for (int l = from; l < m; ++l) {                   // the rest of the window head by head
                const int hl = __builtin_amdgcn_readlane(cur.hi, l), el = __builtin_amdgcn_readlane(cur.end, l);
                s = s + rlf(cur.x, l);
                const double dl = static_cast<double>(s);
                const int fl = __builtin_amdgcn_readlane(cur.flag, l);
                const bool okl = fl == 1 || (fl == 0 && dl >= rl64d(cur.dlo, l) && dl <= rl64d(cur.dhi, l));
                if (__builtin_amdgcn_readfirstlane(okl ? 1 : 0)) {
                    s = s + rlf(cur.dq, l);
                } else {
                    const bool chl = fl == kMwFail && el - hl > 1;
                    chained += chl ? 1 : 0;
                    LO_WALK_TERMS(chl, s = walk_terms(col, hl + 1, el, s));
                    ++fbs;
                }
            }
#ifdef LO_EXACT_STAMPS
            t_slow += __builtin_amdgcn_s_memtime() - t_s0;
#endif
            return;
        }
    };
#undef LO_WALK_TERMS
    // the next window's records in flight; two windows per trip, so the loop carries no register copy of a window
    // whose loads are in flight (a copy would wait for them)
    Win wa = load(0);
    for (int k0 = 0; k0 < total; k0 += 128) {
        const Win wb = load(k0 + 64);
        process(wa, k0);
        if (k0 + 64 >= total) break;
        wa = load(k0 + 128);
        process(wb, k0 + 64);
    }
    if (lane == 0) {
        out[colI] = s;
        if (stats) { stats[3 * colI] = total; stats[3 * colI + 1] = fbs; stats[3 * colI + 2] = chained; }
#ifdef LO_EXACT_STAMPS
        if (st) {                                              // walk statistics summed over columns and iterations
            DevState* w = const_cast<DevState*>(st);
            atomicAdd(&w->dbg[15], static_cast<unsigned long long>(total));
            atomicAdd(&w->dbg[13], static_cast<unsigned long long>(fbs));
            atomicAdd(&w->dbg[12], static_cast<unsigned long long>(chained));
            const unsigned long long t_all = __builtin_amdgcn_s_memtime() - t_begin;
            atomicAdd(&w->dbg[16], t_all);
            atomicMax(&w->dbg[17], t_all);
            atomicAdd(&w->dbg[18], t_ch);
            atomicAdd(&w->dbg[19], t_fs);
            atomicAdd(&w->dbg[20], t_slow - t_ch - t_fs);
            atomicAdd(&w->dbg[21], 1ull);
        }
#endif
    }
}

// Host side: the fp32 sequential sums of ncol columns (col0 + k * ld, n terms each; n_dev: a device-side count <= n_cap
// instead) into out[0, ncol), B sized for n_cap.  stats (nullable): 3 per column.
template <bool FAC>
static void launch_mw_sums_t(const float* col0, int ld, int ncol, int n_cap, const int* n_dev, const DevState* st,
                             const MwBuf& B, float* out, long long* stats, hipStream_t s) {
    const int nc = (n_cap + kMwChunk - 1) / kMwChunk;
    static const bool split = std::getenv("LO_MW_SPLIT") != nullptr;   // A/B: the three-launch classification
    if (nc > 0) {
        if (split) {
            hipLaunchKernelGGL(k_mw_chunk_sums<FAC>, dim3(nc, ncol), dim3(256), 0, s, col0, ld, n_cap, n_dev, st, B);
            hipLaunchKernelGGL(k_mw_drift<FAC>, dim3(nc, ncol), dim3(kMwThreads), 0, s, col0, ld, n_cap, n_dev, st, B);
            hipLaunchKernelGGL((k_mw_classify<false, FAC>), dim3(nc, ncol), dim3(kMwThreads), 0, s, col0, ld, n_cap, n_dev,
                               st, B);
        } else {
            hipLaunchKernelGGL((k_mw_classify<true, FAC>), dim3(nc, ncol), dim3(kMwThreads), 0, s, col0, ld, n_cap, n_dev,
                               st, B);
        }
        hipLaunchKernelGGL(k_mw_compact, dim3(nc, ncol), dim3(256), 0, s, n_cap, n_dev, st, B);
    }
    hipLaunchKernelGGL(k_mw_walk<FAC>, dim3(ncol), dim3(64), 0, s, col0, ld, n_cap, n_dev, st, B, out, stats);
}
// factored: col0 holds the 14 factor rows of the exact terms (k_exact_terms, term-major) and column k is the product
// of rows exact_term_factors(k); else ncol stored columns
void launch_mw_sums(const float* col0, int ld, int ncol, int n_cap, const int* n_dev, const DevState* st, const MwBuf& B,
                    float* out, long long* stats, hipStream_t s, bool factored) {
    if (factored) launch_mw_sums_t<true>(col0, ld, ncol, n_cap, n_dev, st, B, out, stats, s);
    else launch_mw_sums_t<false>(col0, ld, ncol, n_cap, n_dev, st, B, out, stats, s);
}
// Bytes of an MwBuf for ncol columns of up to n_cap terms, and its layout in one allocation.
size_t mw_bytes(int ncol, int n_cap) {
    const size_t nc = static_cast<size_t>(std::max(1, (n_cap + kMwChunk - 1) / kMwChunk));
    const size_t rec = static_cast<size_t>(ncol) * nc * kMwCap, per = static_cast<size_t>(ncol) * nc;
    const size_t crec = static_cast<size_t>(ncol) * (nc * kMwCap + kMwPad);
    return (rec + crec) * (5 * sizeof(int) + 2 * sizeof(double)) + per * (sizeof(int) + 3 * sizeof(double)) +
           static_cast<size_t>(ncol) * sizeof(int) + 20 * 256;
}
MwBuf mw_layout(void* mem, int ncol, int n_cap) {
    MwBuf B{};
    const size_t nc = static_cast<size_t>(std::max(1, (n_cap + kMwChunk - 1) / kMwChunk));
    const size_t rec = static_cast<size_t>(ncol) * nc * kMwCap, per = static_cast<size_t>(ncol) * nc;
    const size_t crec = static_cast<size_t>(ncol) * (nc * kMwCap + kMwPad);
    char* p = static_cast<char*>(mem);
    auto take = [&](size_t bytes) { char* q = p; p += (bytes + 255) / 256 * 256; return q; };
    B.dlo = reinterpret_cast<double*>(take(rec * 8));
    B.dhi = reinterpret_cast<double*>(take(rec * 8));
    B.c_dlo = reinterpret_cast<double*>(take(crec * 8));
    B.c_dhi = reinterpret_cast<double*>(take(crec * 8));
    B.csum = reinterpret_cast<double*>(take(per * 8));
    B.cabs = reinterpret_cast<double*>(take(per * 8));
    B.dcorr = reinterpret_cast<double*>(take(per * 8));
    B.idx = reinterpret_cast<int*>(take(rec * 4));
    B.end = reinterpret_cast<int*>(take(rec * 4));
    B.x = reinterpret_cast<float*>(take(rec * 4));
    B.dq = reinterpret_cast<float*>(take(rec * 4));
    B.flag = reinterpret_cast<int*>(take(rec * 4));
    B.c_idx = reinterpret_cast<int*>(take(crec * 4));
    B.c_end = reinterpret_cast<int*>(take(crec * 4));
    B.c_x = reinterpret_cast<float*>(take(crec * 4));
    B.c_dq = reinterpret_cast<float*>(take(crec * 4));
    B.c_flag = reinterpret_cast<int*>(take(crec * 4));
    B.nh = reinterpret_cast<int*>(take(per * 4));
    B.ntot = reinterpret_cast<int*>(take(static_cast<size_t>(ncol) * 4));
    B.nchunks = static_cast<int>(nc);
    B.cstride = nc * kMwCap + kMwPad;
    return B;
}
// The handed-off chunk values to kMwUnset (once per allocation; k_mw_compact keeps them so).
hipError_t mw_clear(const MwBuf& B, int ncol, hipStream_t s) {
    const size_t per = static_cast<size_t>(ncol) * B.nchunks;
    const char* lo = reinterpret_cast<const char*>(B.csum);
    const char* hi = reinterpret_cast<const char*>(B.dcorr + per);
    return hipMemsetAsync(B.csum, 0xFF, static_cast<size_t>(hi - lo), s);
}

// ---- long mono sums: the iteration-0 scale of scans beyond kExactMaxPoints (lo_seqsum.h MwmBuf) ----
__device__ __forceinline__ bool mwm_skip(const DevState* st, const MwmBuf& B) { return st->done || B.cnt[0] == 0 || B.cnt[1]; }
template <bool SQ>
__device__ __forceinline__ double mwm_term(const double* __restrict__ sorted, int j, int cnt, double m) {
    if (j >= cnt) return 0.0;
    const double v = sorted[j];
    return SQ ? (v - m) * (v - m) : v;
}

// accepted residuals = the finite prefix of the sorted array (cnt[] zeroed by the host first)
__global__ __launch_bounds__(256) void k_mwm_count(const double* __restrict__ sorted, int n, const DevState* st, MwmBuf B) {
    if (st->done) return;
    __shared__ int s_w[4];
    const int i = blockIdx.x * 256 + threadIdx.x;
    const double v = i < n ? sorted[i] : __builtin_inf();
    int fin;
    (void)block_excl_scan<int, 256>(v != __builtin_inf() && !isnan(v) ? 1 : 0, s_w, fin);
    const int nan = __syncthreads_or(isnan(v) ? 1 : 0);
    if (threadIdx.x == 0) {
        if (fin) atomicAdd(&B.cnt[0], fin);
        if (nan) B.cnt[1] = 1;
    }
}

template <bool SQ>
__global__ __launch_bounds__(256) void k_mwm_chunk_sums(const double* __restrict__ sorted, const DevState* st, MwmBuf B) {
    if (mwm_skip(st, B)) return;
    __shared__ double s_w[4];
    const int c = blockIdx.x, tid = threadIdx.x, cnt = B.cnt[0], c0 = c * kMwChunk;
    const double m = SQ ? B.res[0] / cnt : 0.0;
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < kMwChunk / 256; ++k) v += mwm_term<SQ>(sorted, c0 + k * 256 + tid, cnt, m);
    double tot;
    (void)block_excl_scan<double, 256>(v, s_w, tot);
    if (tid == 0) B.csum[c] = tot;
}

struct MwmScratch {
    double wd[kMwWaves];
    long long wl[kMwWaves];
    int wi[kMwWaves];
    int elast[kMwThreads];
    int h_idx[kMwmCap];
    int h_e[kMwmCap];
    int h_c1[kMwmCap];                                         // bit 1: the segment has a tie, bit 0: c1 of its first
    long long h_p[kMwmCap];
};

// A chunk's heads and records (mono_sum_tx's rules, chunk-local: term 0 of every chunk heads a segment, so the
// segmented XOR state starts afresh in every chunk).  Heads: the chunk's first term, every non-zero term whose
// predicted binade differs from its predecessor's, and steps of 2^49 units or more; a halfway tie inside a segment is
// not a head -- its increment follows from the XOR of the increment parities since the segment's previous tie, or, for
// the segment's first tie, from Q's parity at the segment's start (the record's two increments d_0 / d_1).
template <bool SQ>
__global__ __launch_bounds__(kMwThreads) void k_mwm_classify(const double* __restrict__ sorted, const DevState* st, MwmBuf B) {
    if (mwm_skip(st, B)) return;
    __shared__ MwmScratch S;
    const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, cnt = B.cnt[0], c0 = c * kMwChunk, mc = min(kMwChunk, cnt - c0);
    if (mc <= 0) return;
    const double m = SQ ? B.res[0] / cnt : 0.0;
    double t0 = 0.0;
    for (int k = tid; k < c; k += kMwThreads) t0 += B.csum[k];
    double T0;
    (void)block_excl_scan<double, kMwThreads>(t0, S.wd, T0);
    const int base = tid * kMwPT;
    double v[kMwPT];
#pragma unroll
    for (int a = 0; a < kMwPT; ++a) v[a] = base + a < mc ? mwm_term<SQ>(sorted, c0 + base + a, cnt, m) : 0.0;
    double run = 0.0;
#pragma unroll
    for (int a = 0; a < kMwPT; ++a) run += v[a];
    double ttot;
    const double tex = T0 + block_excl_scan<double, kMwThreads>(run, S.wd, ttot);
    S.elast[tid] = binade64(tex + run);
    __syncthreads();
    const int e_in = tid ? S.elast[tid - 1] : kExpNone;
    // predicted binades, term bits, heads
    int E[kMwPT];
    TermBits tb[kMwPT];
    bool hd[kMwPT];
    int nh = 0;
    {
        double tl = 0.0;
        int ep = e_in;
#pragma unroll
        for (int a = 0; a < kMwPT; ++a) {
            tl += v[a];
            const int j = base + a;
            E[a] = binade64(tex + tl);
            const bool act = j < mc && v[a] != 0.0;
            tb[a] = term_bits(v[a], E[a] == kExpNone ? 0 : E[a]);
            hd[a] = j < mc && (j == 0 || (act && (E[a] < -1000 || E[a] != ep || tb[a].f >= (1ll << 49))));
            nh += hd[a] ? 1 : 0;
            ep = E[a];
        }
    }
    auto bits_of = [&](int a) -> int {                          // a term's own 4-bit XOR-scan state (xs_op)
        if (hd[a]) return 1 | 4;
        if (!(base + a < mc && v[a] != 0.0)) return 0;
        if (tb[a].tie) return 1 | 8;
        return static_cast<int>((tb[a].f + tb[a].up) & 1) << 1;
    };
    int xs = 0;
#pragma unroll
    for (int a = 0; a < kMwPT; ++a) xs = xs_op(xs, bits_of(a));
    int xtot = 0;
    const int xex = block_excl_scan_dpp<kMwThreads>(xs | (nh << 4), 0,
                                                    [](int a, int b) { return xs_op(a & 15, b & 15) | (((a >> 4) + (b >> 4)) << 4); },
                                                    S.wi, &xtot);
    const int hbase = xex >> 4, htot = xtot >> 4;
    // increments (a later tie of its segment: f + (XOR ^ f's parity); the first: f, its +1 left to the walk)
    long long inc_tot = 0;
    {
        int st4 = xex & 15;
#pragma unroll
        for (int a = 0; a < kMwPT; ++a) {
            const bool act = base + a < mc && v[a] != 0.0 && !hd[a];
            long long inc = 0;
            if (act) {
                if (tb[a].tie) inc = tb[a].f + ((st4 & 8) ? (((st4 >> 1) ^ static_cast<int>(tb[a].f)) & 1) : 0);
                else inc = tb[a].f + tb[a].up;
            }
            inc_tot += inc;
            st4 = xs_op(st4, bits_of(a));
        }
    }
    for (int k = tid; k < htot; k += kMwThreads) S.h_c1[k] = 0;    // ordered before the records by the scan's barriers
    long long ptot = 0;
    const long long pex = block_excl_scan_dpp<kMwThreads>(inc_tot, 0ll, [](long long a, long long b) { return a + b; }, S.wl, &ptot);
    (void)lane;
    {
        int st4 = xex & 15;
        long long P = pex;
        int hk = hbase;
#pragma unroll
        for (int a = 0; a < kMwPT; ++a) {
            const int j = base + a;
            const bool act = j < mc && v[a] != 0.0 && !hd[a];
            if (hd[a]) { S.h_idx[hk] = j; S.h_e[hk] = E[a]; S.h_p[hk] = P; ++hk; }
            long long inc = 0;
            if (act) {
                if (tb[a].tie) {
                    if (st4 & 8) inc = tb[a].f + (((st4 >> 1) ^ static_cast<int>(tb[a].f)) & 1);
                    else {
                        inc = tb[a].f;
                        if (hk > 0) S.h_c1[hk - 1] = 2 | (((st4 >> 1) ^ static_cast<int>(tb[a].f)) & 1);
                    }
                } else {
                    inc = tb[a].f + tb[a].up;
                }
            }
            P += inc;
            st4 = xs_op(st4, bits_of(a));
        }
    }
    __syncthreads();
    const size_t rb = static_cast<size_t>(c) * kMwmCap;
    for (int k = tid; k < htot; k += kMwThreads) {
        const int hi = S.h_idx[k], E0 = S.h_e[k];
        const bool last = k + 1 >= htot;
        const int hend = last ? mc : S.h_idx[k + 1];
        const long long D = (last ? ptot : S.h_p[k + 1]) - S.h_p[k];
        const int cc = S.h_c1[k];
        const long long d0 = D + ((cc & 2) ? (cc & 1) : 0), d1 = D + ((cc & 2) ? ((cc & 1) ^ 1) : 0);
        int flag = hend > hi + 1 ? 0 : 1;
        double dq = -0.0, dq1 = -0.0, dlo = __builtin_inf(), dhi = -__builtin_inf(), dhi1 = -__builtin_inf();
        if (!flag) {
            if (E0 >= -1000 && D >= 0 && d0 < (1ll << 53) && d1 < (1ll << 53)) {
                const double u = ldexp(1.0, E0 - 52), top = ldexp(1.0, E0 + 1) - u;
                dq = static_cast<double>(d0) * u;
                dq1 = static_cast<double>(d1) * u;
                dlo = ldexp(1.0, E0);
                dhi = top - dq;                                // exact: multiples of u below 2^(E0+1)
                dhi1 = top - dq1;
            } else {
                flag = kMwFail;
            }
        }
        const size_t r = rb + k;
        B.idx[r] = c0 + hi;
        B.end[r] = c0 + hend;
        B.flag[r] = flag;
        B.x[r] = mwm_term<SQ>(sorted, c0 + hi, cnt, m);
        B.dq[r] = dq;
        B.dq1[r] = dq1;
        B.dlo[r] = dlo;
        B.dhi[r] = dhi;
        B.dhi1[r] = dhi1;
    }
    if (tid == 0) B.nh[c] = htot;
}

__global__ __launch_bounds__(256) void k_mwm_compact(const DevState* st, MwmBuf B) {
    if (mwm_skip(st, B)) return;
    __shared__ int s_w[4];
    const int c = blockIdx.x, tid = threadIdx.x, cnt = B.cnt[0], nc = (cnt + kMwChunk - 1) / kMwChunk;
    if (c >= nc) return;
    int before = 0;
    for (int k = tid; k < c; k += 256) before += B.nh[k];
    int off;
    (void)block_excl_scan<int, 256>(before, s_w, off);
    const int h = B.nh[c];
    const size_t src = static_cast<size_t>(c) * kMwmCap;
    for (int k = tid; k < h; k += 256) {
        B.c_idx[off + k] = B.idx[src + k];
        B.c_end[off + k] = B.end[src + k];
        B.c_flag[off + k] = B.flag[src + k];
        B.c_x[off + k] = B.x[src + k];
        B.c_dq[off + k] = B.dq[src + k];
        B.c_dq1[off + k] = B.dq1[src + k];
        B.c_dlo[off + k] = B.dlo[src + k];
        B.c_dhi[off + k] = B.dhi[src + k];
        B.c_dhi1[off + k] = B.dhi1[src + k];
    }
    if (c == nc - 1) {                                         // no-op records after the last head
        if (tid < kMwPad) {
            const int r = off + h + tid;
            B.c_idx[r] = 0; B.c_end[r] = 0; B.c_flag[r] = 1; B.c_x[r] = -0.0; B.c_dq[r] = -0.0; B.c_dq1[r] = -0.0;
            B.c_dlo[r] = 0.0; B.c_dhi[r] = 0.0; B.c_dhi1[r] = 0.0;
        }
        if (tid == 0) B.cnt[2] = off + h;
    }
}

// s + x[j0] + ... + x[j1 - 1] term by term, x = the (squared-deviation) terms, scalar loads as walk_terms
template <bool SQ>
__device__ __forceinline__ double walk_terms_m(const double* __restrict__ sorted, int j0, int j1, int cnt, double m, double s) {
    constexpr int kB = 16;
    j0 = __builtin_amdgcn_readfirstlane(j0);
    j1 = __builtin_amdgcn_readfirstlane(j1);
    const int lane = threadIdx.x & 63;
    int j = j0;
    {                                                          // to a 128-byte boundary: one load per lane
        const int a = min(j1, (j0 + kB - 1) & ~(kB - 1));
        const double v = lane < a - j0 ? mwm_term<SQ>(sorted, j0 + lane, cnt, m) : -0.0;
        for (int l = 0; l < a - j0; ++l) s = s + rl64d(v, l);
        j = a;
    }
    if (j + kB <= j1) {
        double cur[kB], nxt[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) cur[u] = sorted[j + u];
        for (; j + 2 * kB <= j1; j += kB) {
#pragma unroll
            for (int u = 0; u < kB; ++u) nxt[u] = sorted[j + kB + u];
#pragma unroll
            for (int u = 0; u < kB; ++u) s = s + (SQ ? (cur[u] - m) * (cur[u] - m) : cur[u]);
#pragma unroll
            for (int u = 0; u < kB; ++u) cur[u] = nxt[u];
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) s = s + (SQ ? (cur[u] - m) * (cur[u] - m) : cur[u]);
        j += kB;
    }
    {                                                          // the rest (< kB terms): one load per lane
        const double v = lane < j1 - j ? mwm_term<SQ>(sorted, j + lane, cnt, m) : -0.0;
        for (int l = 0; l < j1 - j; ++l) s = s + rl64d(v, l);
    }
    return s;
}

// one wave: every head in order (as k_mw_walk, fp64); the sum into B.res[SQ]; SQ also writes the scale
template <bool SQ>
__global__ __launch_bounds__(64) void k_mwm_walk(const double* __restrict__ sorted, DevState* st, MwmBuf B) {
    if (mwm_skip(st, B)) return;
    const int lane = threadIdx.x, cnt = B.cnt[0], total = B.cnt[2];
    const double m = SQ ? B.res[0] / cnt : 0.0;
    struct Win { int hi, end, flag; double x, dq, dq1, dlo, dhi, dhi1; };
    auto load = [&](int k0) {                                  // records past the last head are no-ops (kMwPad)
        const int k = k0 + lane;
        return Win{B.c_idx[k], B.c_end[k], B.c_flag[k], B.c_x[k], B.c_dq[k], B.c_dq1[k], B.c_dlo[k], B.c_dhi[k], B.c_dhi1[k]};
    };
    // the segment's increments for Q's parity at its start: the low bit of the mantissa of the sum after the head
    auto odd = [](double v) { return (__double2loint(v) & 1) != 0; };
    double s = 0.0;
    int fbs = 0, fbt = 0;
#ifdef LO_EXACT_STAMPS
    const unsigned long long t_start = __builtin_amdgcn_s_memtime();
    unsigned long long t_terms = 0;
#define LO_TT0 const unsigned long long t_a = __builtin_amdgcn_s_memtime();
#define LO_TT1 t_terms += __builtin_amdgcn_s_memtime() - t_a;
#else
#define LO_TT0
#define LO_TT1
#endif
    __shared__ double2 s_xd[64];                               // the window's (x, dq), read back as broadcasts
    __shared__ double s_d1[64];                                //   and dq1
    auto process = [&](const Win& cur, int k0) {
        double rec = 0.0;
        s_xd[lane] = make_double2(cur.x, cur.dq);
        s_d1[lane] = cur.dq1;
        __syncthreads();
        LO_TT0
#pragma unroll
        for (int l = 0; l < 64; ++l) {
            const double2 xd = s_xd[l];
            const double d1 = s_d1[l];
            s = s + xd.x;
            rec = lane == l ? s : rec;
            s = s + (odd(s) ? d1 : xd.y);
        }
        LO_TT1
        __syncthreads();
        const bool ok = cur.flag == 1 || (cur.flag == 0 && rec >= cur.dlo && rec <= (odd(rec) ? cur.dhi1 : cur.dhi));
        const unsigned long long badm = __ballot(!ok);
        if (badm) {
            const int f = __builtin_ctzll(badm);
            s = rl64d(rec, f);                                  // exact: every head before f passed
            s = walk_terms_m<SQ>(sorted, __builtin_amdgcn_readlane(cur.hi, f) + 1, __builtin_amdgcn_readlane(cur.end, f),
                                 cnt, m, s);
            ++fbs;
            fbt += __builtin_amdgcn_readlane(cur.end, f) - __builtin_amdgcn_readlane(cur.hi, f) - 1;
            const int mw = min(64, total - k0);
            for (int l = f + 1; l < mw; ++l) {
                s = s + rl64d(cur.x, l);
                const int fl = __builtin_amdgcn_readlane(cur.flag, l);
                const bool okl = fl == 1 || (fl == 0 && s >= rl64d(cur.dlo, l) && s <= (odd(s) ? rl64d(cur.dhi1, l) : rl64d(cur.dhi, l)));
                if (__builtin_amdgcn_readfirstlane(okl ? 1 : 0)) s = s + (odd(s) ? rl64d(cur.dq1, l) : rl64d(cur.dq, l));
                else {
                    s = walk_terms_m<SQ>(sorted, __builtin_amdgcn_readlane(cur.hi, l) + 1,
                                         __builtin_amdgcn_readlane(cur.end, l), cnt, m, s);
                    ++fbs;
                    fbt += __builtin_amdgcn_readlane(cur.end, l) - __builtin_amdgcn_readlane(cur.hi, l) - 1;
                }
            }
        }
    };
    Win cur = load(0);                                         // the next window's records in flight
    for (int k0 = 0; k0 < total; k0 += 64) {
        const Win nxt = load(k0 + 64);
        process(cur, k0);
        cur = nxt;
    }
    if (lane == 0) {
        B.res[SQ ? 1 : 0] = s;
        if (SQ) st->scale = sqrt(s / cnt) / 6.0;
        (void)fbs;
        (void)fbt;
#ifdef LO_EXACT_STAMPS
        st->dbg[SQ ? 8 : 5] = static_cast<unsigned long long>(total);   // walk statistics of the last scan
        st->dbg[SQ ? 9 : 6] = static_cast<unsigned long long>(fbs);
        st->dbg[SQ ? 10 : 7] = static_cast<unsigned long long>(fbt);
        if (!SQ) { st->dbg[11] = __builtin_amdgcn_s_memtime() - t_start; st->dbg[14] = t_terms; }
#endif
#undef LO_TT0
#undef LO_TT1
    }
}

// a NaN residual: the reference's sums are NaN and so is the scale (k_exact_scale's rule)
__global__ void k_mwm_nan(const double* __restrict__ sorted, DevState* st, MwmBuf B) {
    if (st->done || B.cnt[0] == 0 || !B.cnt[1]) return;      // no correspondence: the PKO launch reports it
    st->scale = __builtin_nan("");
}

void launch_mwm_scale(KParams P, const double* sorted, const MwmBuf& B, hipStream_t s) {
    const int n = P.n, nc = (n + kMwChunk - 1) / kMwChunk;
    (void)hipMemsetAsync(B.cnt, 0, 3 * sizeof(int), s);
    hipLaunchKernelGGL(k_mwm_count, dim3((n + 255) / 256), dim3(256), 0, s, sorted, n, P.st, B);
    hipLaunchKernelGGL(k_mwm_nan, dim3(1), dim3(1), 0, s, sorted, P.st, B);
    hipLaunchKernelGGL(k_mwm_chunk_sums<false>, dim3(nc), dim3(256), 0, s, sorted, P.st, B);
    hipLaunchKernelGGL(k_mwm_classify<false>, dim3(nc), dim3(kMwThreads), 0, s, sorted, P.st, B);
    hipLaunchKernelGGL(k_mwm_compact, dim3(nc), dim3(256), 0, s, P.st, B);
    hipLaunchKernelGGL(k_mwm_walk<false>, dim3(1), dim3(64), 0, s, sorted, P.st, B);
    hipLaunchKernelGGL(k_mwm_chunk_sums<true>, dim3(nc), dim3(256), 0, s, sorted, P.st, B);
    hipLaunchKernelGGL(k_mwm_classify<true>, dim3(nc), dim3(kMwThreads), 0, s, sorted, P.st, B);
    hipLaunchKernelGGL(k_mwm_compact, dim3(nc), dim3(256), 0, s, P.st, B);
    hipLaunchKernelGGL(k_mwm_walk<true>, dim3(1), dim3(64), 0, s, sorted, P.st, B);
}
size_t mwm_bytes(int n_cap) {
    const size_t nc = static_cast<size_t>(std::max(1, (n_cap + kMwChunk - 1) / kMwChunk)), rec = nc * kMwmCap;
    return (2 * rec + kMwPad) * (3 * sizeof(int) + 6 * sizeof(double)) + nc * (sizeof(int) + sizeof(double)) + 64 +
           24 * 256;
}
MwmBuf mwm_layout(void* mem, int n_cap) {
    MwmBuf B{};
    const size_t nc = static_cast<size_t>(std::max(1, (n_cap + kMwChunk - 1) / kMwChunk)), rec = nc * kMwmCap;
    char* p = static_cast<char*>(mem);
    auto take = [&](size_t bytes) { char* q = p; p += (bytes + 255) / 256 * 256; return q; };
    B.x = reinterpret_cast<double*>(take(rec * 8));
    B.dq = reinterpret_cast<double*>(take(rec * 8));
    B.dq1 = reinterpret_cast<double*>(take(rec * 8));
    B.dlo = reinterpret_cast<double*>(take(rec * 8));
    B.dhi = reinterpret_cast<double*>(take(rec * 8));
    B.dhi1 = reinterpret_cast<double*>(take(rec * 8));
    B.c_x = reinterpret_cast<double*>(take((rec + kMwPad) * 8));
    B.c_dq = reinterpret_cast<double*>(take((rec + kMwPad) * 8));
    B.c_dq1 = reinterpret_cast<double*>(take((rec + kMwPad) * 8));
    B.c_dlo = reinterpret_cast<double*>(take((rec + kMwPad) * 8));
    B.c_dhi = reinterpret_cast<double*>(take((rec + kMwPad) * 8));
    B.c_dhi1 = reinterpret_cast<double*>(take((rec + kMwPad) * 8));
    B.csum = reinterpret_cast<double*>(take(nc * 8));
    B.res = reinterpret_cast<double*>(take(16));
    B.idx = reinterpret_cast<int*>(take(rec * 4));
    B.end = reinterpret_cast<int*>(take(rec * 4));
    B.flag = reinterpret_cast<int*>(take(rec * 4));
    B.c_idx = reinterpret_cast<int*>(take((rec + kMwPad) * 4));
    B.c_end = reinterpret_cast<int*>(take((rec + kMwPad) * 4));
    B.c_flag = reinterpret_cast<int*>(take((rec + kMwPad) * 4));
    B.nh = reinterpret_cast<int*>(take(nc * 4));
    B.cnt = reinterpret_cast<int*>(take(16));
    B.nchunks = static_cast<int>(nc);
    return B;
}

// large scans: the fp32 solve of the 43 column sums (launch_mw_sums), as k_exact_solve does it
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
