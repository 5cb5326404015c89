// lo_kernels.hip — HIP kernels of the point-to-plane ICP hot path for gfx950 (MI355X / CDNA4).
//
// One Gauss-Newton iteration of IterativeClosestPointOptimizer::optimize
// (reference src/optimization/IterativeClosestPointOptimizer.cpp:281-449) is four launches on one stream:
//   k_correspond  per point: transform, L1 surfel probe, fp64 residual, accept r <= max_corr
//                 (find_correspondences :587-645); per-wave validity ballots; iteration 0 also the
//                 per-block residual sum / M2 for the normalisation scale (:304-316)
//   k_pko         one workgroup: correspondence count, scale, the reference's PKO sample selection
//                 (std::shuffle(mt19937(42)) reproduced from host tables), k-means + EM GMM fit and the
//                 JS-divergence alpha grid (AdaptiveMEstimator.cpp:243-485, :710-787)
//   k_accumulate  per correspondence: Huber weight, residual, Jacobian, 21+6+1 partial sums; wave shuffle
//                 + LDS tree to one 28-double partial per block (:345-410)
//   k_solve       one workgroup: fixed-order fp64 sum of block partials, pivoted LDLT (:418),
//                 SE3 right-update with SO(3) re-projection (:422-434), convergence flag (:437-448)
// Every kernel first reads DevState::done, so the whole max_iterations sequence is enqueued once and
// converged / failed scans fall through without a host round trip.
//
// Compiled with -ffp-contract=off: the correspondence set and the fp64 residuals are bit-identical to the
// reference's fp32/fp64 expressions (DESIGN.md "fp order").  Sums are fixed-order trees (run-to-run
// deterministic), not the reference's sequential order.
#include "lo_device.h"

#include <cfloat>

namespace lo {

// ====================================================================================================
// k_correspond
// ====================================================================================================
__global__ __launch_bounds__(kBlock) void k_correspond(KParams P, int with_stats) {
    const DevState* st = P.st;
    if (st->done) return;
    __shared__ double s_red[kWavesPerBlock];
    __shared__ int s_cnt[kWavesPerBlock];
    __shared__ double s_mean;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int i = blockIdx.x * kBlock + tid;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = st->pose[k];

    int slot = -1;
    double r = 0.0;
    if (i < P.n) {
        const float x = P.pts[3 * i], y = P.pts[3 * i + 1], z = P.pts[3 * i + 2];
        float wx, wy, wz;
        transform_pt(T, x, y, z, wx, wy, wz);
        const int s = lookup_surfel(P.tab, P.log2cap, P.l1scale, wx, wy, wz);
        if (s >= 0) {
            const Slot sl = P.tab[s];
            r = residual_f64(sl, wx, wy, wz);
            if (!(r > P.maxd)) slot = s;     // reference rejects only residual > max (NaN kept, as :630)
        }
        P.slot[i] = slot;
        if (P.res_dbg) P.res_dbg[i] = slot >= 0 ? r : 0.0;
    }
    const bool valid = slot >= 0;
    const uint64_t m = __ballot(valid);
    if (lane == 0) {
        P.wmask[blockIdx.x * kWavesPerBlock + wid] = m;
        s_cnt[wid] = __popcll(m);
    }
    if (!with_stats) {
        __syncthreads();
        if (tid == 0) {
            int c = 0;
            for (int w = 0; w < kWavesPerBlock; ++w) c += s_cnt[w];
            P.blk_cnt[blockIdx.x] = c;
        }
        return;
    }
    // iteration 0: per-block (count, sum, M2) for a stable fp64 merge of the residual variance
    double v = wave_sum(valid ? r : 0.0);
    if (lane == 0) s_red[wid] = v;
    __syncthreads();
    if (tid == 0) {
        int c = 0;
        double sum = 0.0;
        for (int w = 0; w < kWavesPerBlock; ++w) { c += s_cnt[w]; sum += s_red[w]; }
        P.blk_cnt[blockIdx.x] = c;
        P.blk_sum[blockIdx.x] = sum;
        s_mean = c > 0 ? sum / c : 0.0;
    }
    __syncthreads();
    const double mb = s_mean;
    const double d = valid ? (r - mb) : 0.0;
    v = wave_sum(d * d);
    __syncthreads();
    if (lane == 0) s_red[wid] = v;
    __syncthreads();
    if (tid == 0) {
        double m2 = 0.0;
        for (int w = 0; w < kWavesPerBlock; ++w) m2 += s_red[w];
        P.blk_m2[blockIdx.x] = m2;
    }
}

// ====================================================================================================
// k_pko
// ====================================================================================================
__device__ __forceinline__ int pko_sample(const KParams& P, int n, int s) {
    if (n < P.S) return P.small_perm[P.small_off[n] + s];
    const int mode = (n <= 65535) ? ((n & 1) ? 0 : 1) : 2;
    const int lo0 = P.ev_off[mode * (P.S + 1) + s], hi0 = P.ev_off[mode * (P.S + 1) + s + 1];
    // last event step <= n-1
    int lo = lo0, hi = hi0;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (P.ev_steps[mid] <= n - 1) lo = mid + 1; else hi = mid;
    }
    return lo == lo0 ? P.base[mode * P.S + s] : P.ev_steps[lo - 1];
}

// gaussian_pdf (AdaptiveMEstimator.cpp:675-685)
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

__device__ __forceinline__ double std_max(double a, double b) { return (a < b) ? b : a; }

__global__ __launch_bounds__(kPkoThreads) void k_pko(KParams P, int it) {
    DevState* st = P.st;
    if (st->done) return;
    __shared__ double sh[10240];                 // 80 KB: block prefix (as int) / JS chunk table
    __shared__ double s_sd[kMaxS];
    __shared__ double s_P[100];
    __shared__ double s_js[kMaxAlpha + 1];
    __shared__ double s_red[kPkoThreads / 64];
    __shared__ int s_ired[kPkoThreads / 64];
    __shared__ double s_gmm[3 * kMaxK];
    __shared__ int s_nc;
    __shared__ double s_scale, s_mean;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    constexpr int NW = kPkoThreads / 64;
    int* pre = reinterpret_cast<int*>(sh);

    if (P.direct_res) {
        if (tid == 0) { s_nc = P.n; s_scale = 1.0; }
        __syncthreads();
    } else {
        // ---- 1. exclusive prefix of per-block correspondence counts (rank -> block) + stats merge ----
        const int nb = P.nb;
        const int per = (nb + kPkoThreads - 1) / kPkoThreads;
        const int b0 = min(tid * per, nb), b1 = min(b0 + per, nb);
        int loc = 0;
        double lsum = 0.0;
        for (int b = b0; b < b1; ++b) { loc += P.blk_cnt[b]; if (it == 0) lsum += P.blk_sum[b]; }
        int inc = loc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) { const int t = __shfl_up(inc, o, 64); if (lane >= o) inc += t; }
        if (lane == 63) s_ired[wid] = inc;
        const double ws = wave_sum(lsum);
        if (lane == 0) s_red[wid] = ws;
        __syncthreads();
        if (tid == 0) {
            int run = 0;
            double tot = 0.0;
            for (int w = 0; w < NW; ++w) { const int c = s_ired[w]; s_ired[w] = run; run += c; tot += s_red[w]; }
            s_nc = run;
            s_mean = run > 0 ? tot / run : 0.0;
        }
        __syncthreads();
        int excl = s_ired[wid] + inc - loc;
        for (int b = b0; b < b1; ++b) { pre[b] = excl; excl += P.blk_cnt[b]; }
        if (it == 0) {
            const double mean = s_mean;
            double m2 = 0.0;
            for (int b = b0; b < b1; ++b) {
                const int c = P.blk_cnt[b];
                if (c > 0) { const double dm = P.blk_sum[b] / c - mean; m2 += P.blk_m2[b] + c * (dm * dm); }
            }
            m2 = wave_sum(m2);
            __syncthreads();
            if (lane == 0) s_red[wid] = m2;
            __syncthreads();
            if (tid == 0) {
                double M2 = 0.0;
                for (int w = 0; w < NW; ++w) M2 += s_red[w];
                const double var = s_nc > 0 ? M2 / s_nc : 0.0;
                s_scale = sqrt(var) / 6.0;            // IterativeClosestPointOptimizer.cpp:314-315
                st->scale = s_scale;
            }
        } else if (tid == 0) {
            s_scale = st->scale;
        }
        __syncthreads();
    }
    const int nc = s_nc;
    if (nc < P.min_corr && !P.direct_res) {               // :298-302
        if (tid == 0) { st->status = LO_INSUFFICIENT; st->done = 1; st->n_corr = nc; }
        return;
    }
    if (!P.use_pko || nc == 0) {
        if (tid == 0) { st->alpha = nc == 0 ? 1.0 : P.robust_delta; st->n_corr = nc; }
        return;
    }
    const double scale = s_scale;
    const double sden = std_max(scale, 1e-6);

    // ---- 2. the reference's GMM sample: r_hat[perm_nc[s]], s < min(S, nc) ----
    const int S = min(P.S, nc);
    if (tid < S) {
        const int rank = pko_sample(P, nc, tid);
        double v;
        if (P.direct_res) {
            v = P.direct_res[rank];
        } else {
            int lo = 0, hi = P.nb - 1;                     // last block with pre[b] <= rank
            while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (pre[mid] <= rank) lo = mid; else hi = mid - 1; }
            const int b = lo;
            int k = rank - pre[b];
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
            for (int q = 0; q < 12; ++q) T[q] = st->pose[q];
            float wx, wy, wz;
            transform_pt(T, P.pts[3 * pidx], P.pts[3 * pidx + 1], P.pts[3 * pidx + 2], wx, wy, wz);
            const double r = residual_f64(P.tab[P.slot[pidx]], wx, wy, wz);
            v = r / sden;                                   // :321-326
        }
        s_sd[tid] = v;
    }
    __syncthreads();

    // ---- 3. GMM: k-means init + EM (fit_gmm, AdaptiveMEstimator.cpp:294-485), wave 0 ----
    // Loops run to the compile-time kMaxK with `j < K` guards so every per-component array stays in VGPRs.
    const int K = P.K;
    if (wid == 0) {
        double x[4];
        bool have[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) { const int idx = lane + 64 * q; have[q] = idx < S; x[q] = have[q] ? s_sd[idx] : 0.0; }
        double mu[kMaxK], var[kMaxK], w[kMaxK], cntd[kMaxK];
        const int D = K > 1 ? K - 1 : 1;
#pragma unroll
        for (int j = 0; j < kMaxK; ++j) { mu[j] = (j > 0 && j < K) ? s_sd[P.km_draws[S * D + (j - 1)]] : 0.0; cntd[j] = 0.0; }
        for (int guard = 0; guard < 100000; ++guard) {
            double sums[kMaxK];
#pragma unroll
            for (int j = 0; j < kMaxK; ++j) { sums[j] = 0.0; cntd[j] = 0.0; }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (!have[q]) continue;
                double md = DBL_MAX;
                int ci = 0;
#pragma unroll
                for (int j = 0; j < kMaxK; ++j) if (j < K) { const double d = fabs(x[q] - mu[j]); if (d < md) { md = d; ci = j; } }
#pragma unroll
                for (int j = 0; j < kMaxK; ++j) if (j == ci) { sums[j] += x[q]; cntd[j] += 1.0; }
            }
            bool eq = true;
            double nm[kMaxK];
#pragma unroll
            for (int j = 0; j < kMaxK; ++j) {
                if (j < K) {
                    sums[j] = wave_sum(sums[j]);
                    cntd[j] = wave_sum(cntd[j]);
                }
                nm[j] = (j == 0 || j >= K) ? 0.0 : (cntd[j] > 0.0 ? sums[j] / cntd[j] : 0.0);
                eq = eq && (nm[j] == mu[j]);
            }
            if (eq) break;
#pragma unroll
            for (int j = 0; j < kMaxK; ++j) mu[j] = nm[j];
        }
        double sx = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) if (have[q]) sx += x[q];
        const double mean_of_data = wave_sum(sx) / S;
        double sv = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) if (have[q]) { const double d = x[q] - mean_of_data; sv += d * d; }
        const double iv = wave_sum(sv) / S;
#pragma unroll
        for (int j = 0; j < kMaxK; ++j) { var[j] = iv; w[j] = cntd[j] / static_cast<double>(S); }

        for (int em = 0; em < 100; ++em) {
            double Nk[kMaxK], Sx[kMaxK], resp[4][kMaxK], nrm[kMaxK];
#pragma unroll
            for (int j = 0; j < kMaxK; ++j) { Nk[j] = 0.0; Sx[j] = 0.0; nrm[j] = var[j] <= 0.0 ? 0.0 : 1.0 / sqrt(2.0 * M_PI * var[j]); }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                double sr = 0.0;
#pragma unroll
                for (int j = 0; j < kMaxK; ++j) {
                    double pdf = 0.0;
                    if (var[j] > 0.0) { const double diff = x[q] - mu[j]; pdf = nrm[j] * exp(-0.5 * (diff * diff) / var[j]); }
                    resp[q][j] = w[j] * pdf;
                    if (j < K) sr += resp[q][j];
                }
#pragma unroll
                for (int j = 0; j < kMaxK; ++j) {
                    resp[q][j] /= sr;
                    if (have[q] && j < K) { Nk[j] += resp[q][j]; Sx[j] += resp[q][j] * x[q]; }
                }
            }
            double nmu[kMaxK], nv[kMaxK], nw[kMaxK];
#pragma unroll
            for (int j = 0; j < kMaxK; ++j) {
                if (j < K) { Nk[j] = wave_sum(Nk[j]); Sx[j] = wave_sum(Sx[j]); }
                nw[j] = Nk[j] / static_cast<double>(S);
                nmu[j] = (j == 0 || j >= K) ? 0.0 : Sx[j] / Nk[j];
            }
#pragma unroll
            for (int j = 0; j < kMaxK; ++j) {
                double vv = 0.0;
#pragma unroll
                for (int q = 0; q < 4; ++q) if (have[q]) { const double d = x[q] - nmu[j]; vv += resp[q][j] * d * d; }
                if (j < K) vv = wave_sum(vv);
                nv[j] = std_max(vv / Nk[j], 1e-6);
            }
            double change = 0.0;
#pragma unroll
            for (int j = 1; j < kMaxK; ++j) if (j < K) change += fabs(nmu[j] - mu[j]);
#pragma unroll
            for (int j = 0; j < kMaxK; ++j) { w[j] = nw[j]; mu[j] = nmu[j]; var[j] = nv[j]; }
            if (change < 1e-6) break;
        }
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < kMaxK; ++j) if (j < K) { s_gmm[j] = w[j]; s_gmm[K + j] = mu[j]; s_gmm[2 * K + j] = var[j]; }
        }
    }
    __syncthreads();

    // ---- 4. JS divergence over the alpha grid (calculate_js_divergence :710-787) ----
    const double dr = P.trunc / 100.0;
    if (tid < 100) {
        const double r = dr * (1 + static_cast<double>(tid));
        double Pr = 0.0;
        for (int m = 0; m < K; ++m) Pr += s_gmm[m] * gpdf(r, s_gmm[K + m], s_gmm[2 * K + m]);
        s_P[tid] = Pr + 1e-10;
    }
    __syncthreads();
    const int NA = P.NA;
    for (int c0 = 1; c0 <= NA; c0 += 100) {
        const int na = min(100, NA - c0 + 1);
        for (int idx = tid; idx < na * 100; idx += kPkoThreads) {
            const int a = idx / 100, b = idx - a * 100;
            const double alpha = P.alphas[c0 + a];
            const double pf = P.Z[c0 + a];
            const double r = dr * (1 + static_cast<double>(b));
            const double Pr = s_P[b];
            const double Q = pko_kernel_w(r, alpha, P.pko_cauchy) / (pf + 1e-10) + 1e-10;
            const double M = 0.5 * (Pr + Q);
            sh[idx] = 0.5 * (Pr * log(Pr / M) + Q * log(Q / M));
        }
        __syncthreads();
        if (tid < na) {
            double cost = 0.0, cnt = 0.0;
            for (int b = 0; b < 100; ++b) {
                const double v = sh[tid * 100 + b];
                if (isnan(v)) continue;
                cost += v;
                cnt += 1.0;
            }
            s_js[c0 + tid] = cnt == 0.0 ? DBL_MAX : cost / cnt;
        }
        __syncthreads();
    }
    if (tid == 0) {
        double best_a = P.min_scale, best_c = DBL_MAX;       // calculate_pko_scale_factor :256-275
        for (int i = 1; i <= NA; ++i) if (s_js[i] < best_c) { best_c = s_js[i]; best_a = P.alphas[i]; }
        st->alpha = best_a;
        st->n_corr = nc;
        for (int j = 0; j < 3 * K; ++j) st->gmm_out[j] = s_gmm[j];
    }
}

// ====================================================================================================
// k_accumulate
// ====================================================================================================
__global__ __launch_bounds__(kBlock) void k_accumulate(KParams P) {
    const DevState* st = P.st;
    if (st->done) return;
    __shared__ float s_acc[kWavesPerBlock][kNE];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int i = blockIdx.x * kBlock + tid;
    float acc[kNE];
#pragma unroll
    for (int k = 0; k < kNE; ++k) acc[k] = 0.0f;
    const int s = (i < P.n) ? P.slot[i] : -1;
    if (s >= 0) {
        float T[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
        const double scale = st->scale;
        const float dl = static_cast<float>(st->alpha);
        const float px = P.pts[3 * i], py = P.pts[3 * i + 1], pz = P.pts[3 * i + 2];
        const Slot sl = P.tab[s];
        float wx, wy, wz;
        transform_pt(T, px, py, pz, wx, wy, wz);
        const double r = residual_f64(sl, wx, wy, wz);
        const float nres = static_cast<float>(r / std_max(scale, 1e-6));          // :374
        // p_world = R p + t (Matrix3f * Vector3f, :368), residual n.(p_w - q) in fp32 (:371)
        const float qx = dot3f(T[0], T[1], T[2], px, py, pz) + T[3];
        const float qy = dot3f(T[4], T[5], T[6], px, py, pz) + T[7];
        const float qz = dot3f(T[8], T[9], T[10], px, py, pz) + T[11];
        const float n0 = sl.n[0], n1 = sl.n[1], n2 = sl.n[2];
        const float res = dot3f(n0, n1, n2, qx - sl.c[0], qy - sl.c[1], qz - sl.c[2]);
        // J = [n^T R, -n^T R [p]x] (:376-386)
        float J[6];
        J[0] = dot3f(n0, n1, n2, T[0], T[4], T[8]);
        J[1] = dot3f(n0, n1, n2, T[1], T[5], T[9]);
        J[2] = dot3f(n0, n1, n2, T[2], T[6], T[10]);
        const float a0 = dot3f(-n0, -n1, -n2, T[0], T[4], T[8]);
        const float a1 = dot3f(-n0, -n1, -n2, T[1], T[5], T[9]);
        const float a2 = dot3f(-n0, -n1, -n2, T[2], T[6], T[10]);
        J[3] = dot3f(a0, a1, a2, 0.0f, pz, -py);
        J[4] = dot3f(a0, a1, a2, -pz, 0.0f, px);
        J[5] = dot3f(a0, a1, a2, py, -px, 0.0f);
        float w = 1.0f;
        if (P.robust) {                                                             // :389-404
            const float an = fabsf(nres);
            if (P.cauchy_loss) { const float ratio = an / dl; w = 1.0f / (1.0f + ratio * ratio); }
            else if (an > dl) w = dl / an;
        }
        int k = 0;
#pragma unroll
        for (int rr = 0; rr < 6; ++rr) {
            const float wJ = w * J[rr];
#pragma unroll
            for (int c = 0; c <= rr; ++c) acc[k++] += wJ * J[c];
        }
        const float wr = w * res;
#pragma unroll
        for (int j = 0; j < 6; ++j) acc[21 + j] += wr * J[j];
        acc[27] += wr * res;
    }
#pragma unroll
    for (int k = 0; k < kNE; ++k) {
        const float v = wave_sum(acc[k]);
        if (lane == 0) s_acc[wid][k] = v;
    }
    __syncthreads();
    if (tid < kNE) {
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < kWavesPerBlock; ++w) v += static_cast<double>(s_acc[w][tid]);
        P.blk_part[static_cast<size_t>(blockIdx.x) * kNE + tid] = v;
    }
}

// ====================================================================================================
// k_solve
// ====================================================================================================
__device__ void mul33f(const float* A, const float* B, float* C) {   // Matrix3f * Matrix3f, row-major
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) C[r * 3 + c] = dot3f(A[r * 3], A[r * 3 + 1], A[r * 3 + 2], B[c], B[3 + c], B[6 + c]);
}

// SO3(const Matrix3f&) projects onto SO(3) with an fp32 JacobiSVD (MathUtils.cpp:86-99).  Here: the
// orthogonal polar factor U V^T computed in fp64 by Newton's iteration X <- (X + X^-T)/2, then rounded.
__device__ void so3_project(const float* Min, float* Rout) {
    double X[9];
    for (int k = 0; k < 9; ++k) X[k] = Min[k];
    for (int itn = 0; itn < 6; ++itn) {
        const double c00 = X[4] * X[8] - X[5] * X[7], c01 = X[5] * X[6] - X[3] * X[8], c02 = X[3] * X[7] - X[4] * X[6];
        const double c10 = X[2] * X[7] - X[1] * X[8], c11 = X[0] * X[8] - X[2] * X[6], c12 = X[1] * X[6] - X[0] * X[7];
        const double c20 = X[1] * X[5] - X[2] * X[4], c21 = X[2] * X[3] - X[0] * X[5], c22 = X[0] * X[4] - X[1] * X[3];
        const double det = X[0] * c00 + X[1] * c01 + X[2] * c02;
        if (!(det > 0.0)) break;
        const double id = 1.0 / det;
        const double C[9] = {c00, c01, c02, c10, c11, c12, c20, c21, c22};   // cofactor = det * X^-T
        for (int k = 0; k < 9; ++k) X[k] = 0.5 * (X[k] + C[k] * id);
    }
    for (int k = 0; k < 9; ++k) Rout[k] = static_cast<float>(X[k]);
}

// SO3::Exp (MathUtils.cpp:23-39), kEps = 1e-6f
__device__ void so3_exp(const float* w, float* R) {
    const float theta = sqrtf(dot3f(w[0], w[1], w[2], w[0], w[1], w[2]));
    float M[9];
    if (theta < 1e-6f) {
        M[0] = 1.0f; M[1] = -w[2]; M[2] = w[1];
        M[3] = w[2]; M[4] = 1.0f; M[5] = -w[0];
        M[6] = -w[1]; M[7] = w[0]; M[8] = 1.0f;
        so3_project(M, R);
        return;
    }
    const float ti = 1.0f / theta;
    const float k0 = w[0] * ti, k1 = w[1] * ti, k2 = w[2] * ti;
    const float K[9] = {0.0f, -k2, k1, k2, 0.0f, -k0, -k1, k0, 0.0f};
    const float s = sinf(theta), omc = 1.0f - cosf(theta);
    float sK[9], KK[9];
    for (int k = 0; k < 9; ++k) sK[k] = omc * K[k];
    mul33f(sK, K, KK);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) M[r * 3 + c] = ((r == c ? 1.0f : 0.0f) + s * K[r * 3 + c]) + KK[r * 3 + c];
    so3_project(M, R);
}

// H.ldlt().solve(b): Eigen's pivoted LDLT (LDLT.h ldlt_inplace<Lower>::unblocked / _solve_impl) in fp64
__device__ void ldlt6_solve(const double* Hin, const double* b, double* x) {
    double m[36];
    for (int k = 0; k < 36; ++k) m[k] = Hin[k];
    int tr[6];
    double temp[6];
    for (int k = 0; k < 6; ++k) {
        int big = k;
        double bv = fabs(m[k * 7]);
        for (int i = k + 1; i < 6; ++i) if (fabs(m[i * 7]) > bv) { bv = fabs(m[i * 7]); big = i; }
        tr[k] = big;
        if (k != big) {
            for (int j = 0; j < k; ++j) { const double t = m[k * 6 + j]; m[k * 6 + j] = m[big * 6 + j]; m[big * 6 + j] = t; }
            for (int i = big + 1; i < 6; ++i) { const double t = m[i * 6 + k]; m[i * 6 + k] = m[i * 6 + big]; m[i * 6 + big] = t; }
            { const double t = m[k * 7]; m[k * 7] = m[big * 7]; m[big * 7] = t; }
            for (int i = k + 1; i < big; ++i) { const double t = m[i * 6 + k]; m[i * 6 + k] = m[big * 6 + i]; m[big * 6 + i] = t; }
        }
        if (k > 0) {
            for (int j = 0; j < k; ++j) temp[j] = m[j * 7] * m[k * 6 + j];
            double acc = 0.0;
            for (int j = 0; j < k; ++j) acc += m[k * 6 + j] * temp[j];
            m[k * 7] -= acc;
            for (int i = k + 1; i < 6; ++i) {
                double a = 0.0;
                for (int j = 0; j < k; ++j) a += m[i * 6 + j] * temp[j];
                m[i * 6 + k] -= a;
            }
        }
        const double akk = m[k * 7];
        const bool valid = fabs(akk) > 0.0;
        if (k == 0 && !valid) { for (int i = 0; i < 6; ++i) x[i] = 0.0; return; }
        if (valid) for (int i = k + 1; i < 6; ++i) m[i * 6 + k] /= akk;
    }
    double d[6];
    for (int i = 0; i < 6; ++i) d[i] = b[i];
    for (int k = 0; k < 6; ++k) if (tr[k] != k) { const double t = d[k]; d[k] = d[tr[k]]; d[tr[k]] = t; }
    for (int i = 0; i < 6; ++i) { double a = 0.0; for (int j = 0; j < i; ++j) a += m[i * 6 + j] * d[j]; d[i] -= a; }
    for (int i = 0; i < 6; ++i) { if (fabs(m[i * 7]) > DBL_MIN) d[i] /= m[i * 7]; else d[i] = 0.0; }
    for (int i = 5; i >= 0; --i) { double a = 0.0; for (int j = i + 1; j < 6; ++j) a += m[j * 6 + i] * d[j]; d[i] -= a; }
    for (int k = 5; k >= 0; --k) if (tr[k] != k) { const double t = d[k]; d[k] = d[tr[k]]; d[tr[k]] = t; }
    for (int i = 0; i < 6; ++i) x[i] = d[i];
}

__global__ __launch_bounds__(256) void k_solve(KParams P, int it, int ne_only) {
    DevState* st = P.st;
    if (st->done) return;
    __shared__ double part[8][kNE];
    __shared__ double tot[kNE];
    const int tid = threadIdx.x;
    if (tid < 8 * kNE) {
        const int k = tid % kNE, q = tid / kNE;
        double s = 0.0;
        for (int b = q; b < P.nb; b += 8) s += P.blk_part[static_cast<size_t>(b) * kNE + k];
        part[q][k] = s;
    }
    __syncthreads();
    if (tid < kNE) {
        double s = 0.0;
        for (int q = 0; q < 8; ++q) s += part[q][tid];
        tot[tid] = s;
    }
    __syncthreads();
    if (tid != 0) return;

    double H[36], g[6];
    int k = 0;
    for (int r = 0; r < 6; ++r)
        for (int c = 0; c <= r; ++c) { H[r * 6 + c] = tot[k]; H[c * 6 + r] = tot[k]; ++k; }
    for (int j = 0; j < 6; ++j) g[j] = tot[21 + j];
    const double cost = tot[27];
    if (ne_only) {
        for (int q = 0; q < 36; ++q) st->H_out[q] = H[q];
        for (int j = 0; j < 6; ++j) st->g_out[j] = g[j];
        st->cost_out = cost;
        return;
    }
    double mg[6], dd[6];
    for (int j = 0; j < 6; ++j) mg[j] = -g[j];
    ldlt6_solve(H, mg, dd);                                           // :418
    float delta[6];
    for (int j = 0; j < 6; ++j) delta[j] = static_cast<float>(dd[j]);
    const float dt[3] = {delta[0], delta[1], delta[2]}, dw[3] = {delta[3], delta[4], delta[5]};

    float R[9], t[3];
    for (int r = 0; r < 3; ++r) { for (int c = 0; c < 3; ++c) R[r * 3 + c] = st->pose[r * 4 + c]; t[r] = st->pose[r * 4 + 3]; }
    float Rd[9];
    if (sqrtf(dot3f(dw[0], dw[1], dw[2], dw[0], dw[1], dw[2])) < 1e-10f) {   // :427-431
        for (int q = 0; q < 9; ++q) Rd[q] = (q % 4 == 0) ? 1.0f : 0.0f;
    } else {
        so3_exp(dw, Rd);
    }
    float M[9], Rn[9];
    mul33f(R, Rd, M);                                                 // SE3::operator* (MathUtils.h:144-147)
    so3_project(M, Rn);
    float tn[3];
    for (int r = 0; r < 3; ++r) tn[r] = t[r] + dot3f(R[r * 3], R[r * 3 + 1], R[r * 3 + 2], dt[0], dt[1], dt[2]);
    for (int r = 0; r < 3; ++r) { for (int c = 0; c < 3; ++c) st->pose[r * 4 + c] = Rn[r * 3 + c]; st->pose[r * 4 + 3] = tn[r]; }

    const float tdel = sqrtf(dot3f(dt[0], dt[1], dt[2], dt[0], dt[1], dt[2]));
    const float rdel = sqrtf(dot3f(dw[0], dw[1], dw[2], dw[0], dw[1], dw[2]));
    lo_iter_log& L = st->logs[it];
    for (int q = 0; q < 12; ++q) L.pose[q] = st->pose[q];
    L.n_corr = st->n_corr;
    L.scale = st->scale;
    L.alpha = st->alpha;
    L.cost = static_cast<float>(cost);
    k = 0;
    for (int r = 0; r < 6; ++r) for (int c = r; c < 6; ++c) L.H[k++] = static_cast<float>(H[r * 6 + c]);
    for (int j = 0; j < 6; ++j) { L.g[j] = static_cast<float>(g[j]); L.delta[j] = delta[j]; }
    st->iter = it + 1;
    if (tdel < P.tol_t && rdel < P.tol_r) st->done = 1;               // :443-448
}

}  // namespace lo
