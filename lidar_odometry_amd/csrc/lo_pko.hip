// lo_pko.hip — PKO adaptive Huber scale (AdaptiveMEstimator::calculate_scale_factor) on the device.
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
// results, no inter-workgroup traffic) with one sample per lane over NW = ceil(S/64) waves and ONE LDS
// exchange + barrier per EM / k-means iteration; afterwards workgroup g evaluates the JS divergence for
// alphas g+1, g+1+G, ... and writes them to global memory.  The argmin over the grid (first strict minimum,
// as the reference loop) is taken by the consumers (k_accumulate / k_pko_finish) after the kernel boundary,
// so no in-launch hand-off is needed.
#include "lo_device.h"

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

__device__ __forceinline__ double pko_kernel_w(double r, double d, int cauchy) {   // :128-156
    if (!cauchy) { const double a = fabs(r); return a <= d ? 1.0 : d / a; }
    const double e2 = r * r, d2 = d * d;
    return d2 / (d2 + e2);
}

// Diagnostic build only (-DLO_PKO_STAMPS): workgroup 0 / thread 0 stores s_memtime at phase boundaries
// into DevState::dbg (never read by any other code; the real kernel executes no stamp).
#ifdef LO_PKO_STAMPS
#define LO_STAMP(dbg, i) do { if ((dbg) && threadIdx.x == 0) (dbg)[i] = __builtin_amdgcn_s_memtime(); } while (0)
#define LO_COUNT(dbg, i, v) do { if ((dbg) && threadIdx.x == 0) (dbg)[i] = (v); } while (0)
#else
#define LO_STAMP(dbg, i) do { } while (0)
#define LO_COUNT(dbg, i, v) do { } while (0)
#endif

// Block-wide sums of NV <= 8 values per thread.  Intra-wave step is a transposed reduction: every lane
// stores its NV values to its wave's LDS tile, lane l then adds the 8 entries [l>>3][8*(l&7) .. +7] and
// three DPP steps finish each 8-lane group, so value q's wave total sits in lanes 8q..8q+7 (~45
// instructions instead of NV x 6 DPP rounds).  Per-wave totals go through one more LDS tile and ONE
// __syncthreads; the sum over waves is in fixed order.  part[] is double-buffered by the parity bit.
template <int NW>
struct PkoScratch {
    double tile[NW][8][64];
    double part[2][NW][8];
};

template <int NW, int NV>
__device__ __forceinline__ void block_totals(double (&v)[NV], PkoScratch<NW>* sc, int& buf) {
    static_assert(NV <= 8, "transposed reduction handles up to 8 values");
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < NV; ++q) sc->tile[wid][q][lane] = v[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int q = lane >> 3, c = (lane & 7) * 8;
    double t = 0.0;
    if (q < NV) {
        const double* row = &sc->tile[wid][q][c];
        const double a0 = row[0] + row[1], a1 = row[2] + row[3], a2 = row[4] + row[5], a3 = row[6] + row[7];
        t = (a0 + a1) + (a2 + a3);
    }
    t += dpp64<0xB1, 0xf>(t);    // quad_perm [1,0,3,2]
    t += dpp64<0x4E, 0xf>(t);    // quad_perm [2,3,0,1]
    t += dpp64<0x141, 0xf>(t);   // row_half_mirror: 8-lane group total in every lane of the group
    if (lane < NV * 8 && (lane & 7) == 0) sc->part[buf][wid][lane >> 3] = t;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double u = sc->part[buf][0][k];
#pragma unroll
        for (int w = 1; w < NW; ++w) u += sc->part[buf][w][k];
        v[k] = u;
    }
    buf ^= 1;
}

// fit_gmm (AdaptiveMEstimator.cpp:294-485) on S <= 64*NW samples held one per thread.
// The E-step constants w_j / sqrt(2 pi var_j) and 0.5 / var_j are formed once per EM iteration, reciprocals
// are Newton-refined hardware estimates and sums are trees: results move by a few ulp against the
// reference's sequential evaluation.  The device PKO is checked for identical alpha against the reference's
// golden vectors (tests/test_gpu_parity.py::test_pko_alpha_matches_reference_golden).
template <int NW, int K>
__device__ void gmm_fit(const double* s_sd, int S, const int32_t* draws, PkoScratch<NW>* sc, double* gmm,
                        unsigned long long* dbg) {
    static_assert(3 * K - 1 <= 8 && 2 * K - 1 <= 8, "partials");
    const int tid = threadIdx.x;
    const bool have = tid < S;
    const double x = have ? s_sd[tid] : 0.0;
    int buf = 0;
    double mu[K], cnt[K];
    mu[0] = 0.0;
#pragma unroll
    for (int j = 1; j < K; ++j) mu[j] = s_sd[draws[j - 1]];
#pragma unroll
    for (int j = 0; j < K; ++j) cnt[j] = 0.0;

    // ---- k-means until the means repeat exactly (:351-389) ----
    for (int guard = 0; guard < 100000; ++guard) {
        double md = DBL_MAX;
        int ci = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) { const double d = fabs(x - mu[j]); if (d < md) { md = d; ci = j; } }
        double v[2 * K - 1];                               // counts 0..K-1, sums 1..K-1
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const bool mine = have && ci == j;
            v[j] = mine ? 1.0 : 0.0;
            if (j > 0) v[K + j - 1] = mine ? x : 0.0;
        }
        block_totals<NW, 2 * K - 1>(v, sc, buf);
        bool eq = true;
        double nm[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            nm[j] = (j == 0) ? 0.0 : (v[j] > 0.0 ? v[K + j - 1] / v[j] : 0.0);
            eq = eq && (nm[j] == mu[j]);
            cnt[j] = v[j];
        }
        LO_COUNT(dbg, 9, guard + 1);
        if (eq) break;
#pragma unroll
        for (int j = 0; j < K; ++j) mu[j] = nm[j];
    }
    LO_STAMP(dbg, 3);
    // ---- initial variance of the sample (:392-399), weights from cluster sizes (:402-410) ----
    double m1[1] = {have ? x : 0.0};
    block_totals<NW, 1>(m1, sc, buf);
    const double mean = m1[0] / S;
    double m2[1] = {have ? (x - mean) * (x - mean) : 0.0};
    block_totals<NW, 1>(m2, sc, buf);
    const double iv = m2[0] / S;
    const double invS = 1.0 / static_cast<double>(S);
    double w[K], var[K], ca[K], cb[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        var[j] = iv;
        w[j] = cnt[j] / static_cast<double>(S);
        ca[j] = w[j] * rsq64(2.0 * M_PI * iv);
        cb[j] = 0.5 * rcp64(iv);
    }
    LO_STAMP(dbg, 4);

    // ---- EM, <= 100 iterations, tolerance 1e-6 on the summed |d mean| of components >= 1 (:413-484) ----
    // One reduction round per iteration: N_j, sum r x (j >= 1) and sum r (x - c_j)^2 about the previous
    // mean c_j; var_j = sum r (x - c_j)^2 / N_j - (mu_j - c_j)^2 (the two-pass sum up to rounding).
    for (int em = 0; em < 100; ++em) {
        double p[K], d[K], sr = 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            d[j] = x - mu[j];
            const double e = exp(-((d[j] * d[j]) * cb[j]));
            p[j] = (var[j] <= 0.0) ? 0.0 : ca[j] * e;      // gaussian_pdf returns 0 for var <= 0
            sr += p[j];
        }
        const double isr = rcp64(sr);
        double v[3 * K - 1];                               // N_j | sum r x (j>=1) | sum r d^2
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const double r = p[j] * isr;
            v[j] = have ? r : 0.0;
            if (j > 0) v[K + j - 1] = have ? r * x : 0.0;
            v[2 * K - 1 + j] = have ? (r * d[j]) * d[j] : 0.0;
        }
        block_totals<NW, 3 * K - 1>(v, sc, buf);
        double change = 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const double Nk = v[j];
            const double iN = rcp64(Nk);
            const double nmu = (j == 0) ? 0.0 : v[K + j - 1] * iN;
            const double dm = nmu - mu[j];
            double nv = v[2 * K - 1 + j] * iN - dm * dm;
            nv = (nv < 1e-6) ? 1e-6 : nv;                  // std::max(nv, 1e-6), NaN preserved
            if (j >= 1) change += fabs(dm);
            w[j] = Nk * invS;
            mu[j] = nmu;
            var[j] = nv;
            ca[j] = w[j] * rsq64(2.0 * M_PI * nv);
            cb[j] = 0.5 * rcp64(nv);
        }
        LO_COUNT(dbg, 8, em + 1);
        if (change < 1e-6) break;
    }
    LO_STAMP(dbg, 5);
    if (tid == 0) {
#pragma unroll
        for (int j = 0; j < K; ++j) { gmm[j] = w[j]; gmm[K + j] = mu[j]; gmm[2 * K + j] = var[j]; }
    }
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void k_pko_t(KParams P, int it) {
    constexpr int NT = NW * 64;
    DevState* st = P.st;
    if (st->done) return;
    unsigned long long* dbg = nullptr;
#ifdef LO_PKO_STAMPS
    if (blockIdx.x == 0) dbg = st->dbg;
#endif
    LO_STAMP(dbg, 0);
    __shared__ int s_pre[kMaxBlocks];                // 64 KB: exclusive prefix of block counts
    __shared__ double s_sd[64 * NW];
    __shared__ PkoScratch<NW> s_scratch;
    __shared__ double s_gmm[3 * kMaxK];
    __shared__ double s_P[100];
    __shared__ double s_jsd[kPkoAlphaPerWG][100];
    __shared__ int s_iscan[NW];
    __shared__ double s_dscan[NW];
    __shared__ int s_nc;
    __shared__ double s_scale, s_mean;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const bool lead = blockIdx.x == 0;

    // ---- 1. n_c, rank -> block prefix, iteration-0 scale ----
    if (P.direct_res) {
        if (tid == 0) { s_nc = P.n; s_scale = 1.0; }
        __syncthreads();
    } else {
        const int nb = P.nb;
        // (a) coalesced pass: block counts -> LDS, total count / residual sum
        int cnt = 0;
        double lsum = 0.0;
#pragma unroll 4
        for (int b = tid; b < nb; b += NT) {
            const int c = P.blk_cnt[b];
            s_pre[b] = c;
            cnt += c;
            if (it == 0) lsum += P.blk_sum[b];
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
        if (it == 0) {
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
            if (it == 0) {
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
    const int nc = s_nc;
    if (!P.direct_res && nc < P.min_corr) {                     // :298-302
        if (lead && tid == 0) { st->status = LO_INSUFFICIENT; st->done = 1; st->n_corr = nc; }
        return;
    }
    if (lead && tid == 0) st->n_corr = nc;
    if (!P.use_pko || nc == 0) return;                          // consumers use robust_loss_delta / 1.0
    const double scale = s_scale;
    const double sden = (scale < 1e-6) ? 1e-6 : scale;         // std::max(scale, 1e-6)
    LO_STAMP(dbg, 1);

    // ---- 2. the reference's GMM sample ----
    const int S = min(P.S, nc);
    if (tid < S) {
        const int rank = pko_sample(P, nc, tid);
        double v;
        if (P.direct_res) {
            v = P.direct_res[rank];
        } else {
            int lo = 0, hi = P.nb - 1;                          // last block with prefix <= rank
            while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (s_pre[mid] <= rank) lo = mid; else hi = mid - 1; }
            const int b = lo;
            int k = rank - s_pre[b];
            int w = 0;
            uint64_t mk = 0;
            for (; w < kWavesPerBlock; ++w) {
                mk = P.wmask[b * kWavesPerBlock + w];
                const int c = __popcll(mk);
                if (k < c) break;
                k -= c;
            }
            for (int q = 0; q < k; ++q) mk &= mk - 1;
            const int bit = __ffsll(static_cast<unsigned long long>(mk)) - 1;
            const int pidx = b * kBlock + w * kWave + bit;
            float T[12];
#pragma unroll
            for (int q = 0; q < 12; ++q) T[q] = st->pose[q];
            float wx, wy, wz;
            transform_pt(T, P.pts[3 * pidx], P.pts[3 * pidx + 1], P.pts[3 * pidx + 2], wx, wy, wz);
            v = residual_f64(P.tab[P.slot[pidx]], wx, wy, wz) / sden;   // :321-326
        }
        s_sd[tid] = v;
    }
    __syncthreads();
    LO_STAMP(dbg, 2);

    // ---- 3. GMM ----
    const int D = P.K > 1 ? P.K - 1 : 1;
    const int32_t* draws = P.km_draws + S * D;
    switch (P.K) {
        case 1: gmm_fit<NW, 1>(s_sd, S, draws, &s_scratch, s_gmm, dbg); break;
        case 2: gmm_fit<NW, 2>(s_sd, S, draws, &s_scratch, s_gmm, dbg); break;
        default: gmm_fit<NW, 3>(s_sd, S, draws, &s_scratch, s_gmm, dbg); break;
    }
    __syncthreads();
    if (lead && tid < 3 * P.K) st->gmm_out[tid] = s_gmm[tid];

    // ---- 4. JS divergence for this workgroup's alphas (calculate_js_divergence :710-787) ----
    const int K = P.K;
    const double dr = P.trunc / 100.0;
    for (int b = tid; b < 100; b += NT) {
        const double r = dr * (1 + static_cast<double>(b));
        double Pr = 0.0;
        for (int m = 0; m < K; ++m) Pr += s_gmm[m] * gpdf(r, s_gmm[K + m], s_gmm[2 * K + m]);
        s_P[b] = Pr + 1e-10;
    }
    __syncthreads();
    const int G = gridDim.x;
    for (int a0 = 1 + blockIdx.x; a0 <= P.NA; a0 += G * kPkoAlphaPerWG) {
        for (int idx = tid; idx < kPkoAlphaPerWG * 100; idx += NT) {
            const int a = idx / 100, b = idx - a * 100;
            const int ai = a0 + a * G;
            if (ai > P.NA) continue;
            const double alpha = P.alphas[ai];
            const double pf = P.Z[ai];
            const double r = dr * (1 + static_cast<double>(b));
            const double Pr = s_P[b];
            const double Q = pko_kernel_w(r, alpha, P.pko_cauchy) / (pf + 1e-10) + 1e-10;
            const double M = 0.5 * (Pr + Q);
            s_jsd[a][b] = 0.5 * (Pr * log(Pr / M) + Q * log(Q / M));
        }
        __syncthreads();
        if (tid < kPkoAlphaPerWG) {
            const int ai = a0 + tid * G;
            if (ai <= P.NA) {
                double cost = 0.0, cnt = 0.0;                    // sequential, bin order, NaN skipped
                for (int b = 0; b < 100; ++b) {
                    const double v = s_jsd[tid][b];
                    if (isnan(v)) continue;
                    cost += v;
                    cnt += 1.0;
                }
                P.js[ai] = cnt == 0.0 ? DBL_MAX : cost / cnt;
            }
        }
        __syncthreads();
    }
    LO_STAMP(dbg, 6);
}

template __global__ void k_pko_t<2>(KParams, int);
template __global__ void k_pko_t<4>(KParams, int);

// PKO-only entry point: argmin of the JS grid -> DevState::alpha (lo_pko_scale_factor).
__global__ void k_pko_finish(KParams P) {
    DevState* st = P.st;
    const double a = pko_select_alpha(P);
    if (threadIdx.x == 0) st->alpha = a;
}

}  // namespace lo
