// lo_solve.h — the GN solve shared by the per-point kernels (lo_kernels.hip) and the KDTree kernels
// (lo_kdtree.hip, k_solve_knn): fixed-order sum of the block partials, pivoted LDLT, SE3 update with SO(3)
// re-projection and the convergence test (IterativeClosestPointOptimizer.cpp:417-449).
#pragma once
#include <cfloat>

#include "lo_device.h"

namespace lo {

__device__ inline void mul33f(const float* A, const float* B, float* C) {   // Matrix3f * Matrix3f, row-major
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) C[r * 3 + c] = dot3f(A[r * 3], A[r * 3 + 1], A[r * 3 + 2], B[c], B[3 + c], B[6 + c]);
}

// SO3(const Matrix3f&) projects onto SO(3) with an fp32 JacobiSVD (MathUtils.cpp:86-99).  Here: the
// orthogonal polar factor U V^T computed in fp64 by Newton's iteration X <- (X + X^-T)/2, then rounded.
__device__ inline void so3_project(const float* Min, float* Rout) {
    double X[9];
    for (int k = 0; k < 9; ++k) X[k] = Min[k];
    // Newton's polar iteration converges quadratically; inputs are orthonormal to fp32 rounding (~1e-7), so
    // three steps reach the fp64 fixed point (1e-7 -> 1e-14 -> fp64 eps)
    for (int itn = 0; itn < 3; ++itn) {
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

// SO3::Exp (MathUtils.cpp:23-39), kEps = 1e-6f.  The reference re-projects Exp's matrix with an fp32 JacobiSVD
// (SO3(const Matrix3f&), :86-99) and again after R * Exp; here only the product is projected -- Exp's output is
// orthonormal to fp32 rounding, so the two orders agree to ~1e-7, far inside the 1e-4 pose tolerance.
__device__ inline void so3_exp(const float* w, float* R) {
    const float theta = sqrtf(dot3f(w[0], w[1], w[2], w[0], w[1], w[2]));
    float M[9];
    if (theta < 1e-6f) {
        M[0] = 1.0f; M[1] = -w[2]; M[2] = w[1];
        M[3] = w[2]; M[4] = 1.0f; M[5] = -w[0];
        M[6] = -w[1]; M[7] = w[0]; M[8] = 1.0f;
        for (int k = 0; k < 9; ++k) R[k] = M[k];
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
        for (int c = 0; c < 3; ++c) R[r * 3 + c] = ((r == c ? 1.0f : 0.0f) + s * K[r * 3 + c]) + KK[r * 3 + c];
}

// H.ldlt().solve(b): Eigen's pivoted LDLT (LDLT.h ldlt_inplace<Lower>::unblocked / _solve_impl) in fp64.
// Fully unrolled; the data-dependent pivot swaps are unrolled selects so the matrix stays in VGPRs.
__device__ __forceinline__ void dswap(double& a, double& b) { const double t = a; a = b; b = t; }

__device__ inline void ldlt6_solve(const double* Hin, const double* b, double* x) {
    double m[6][6];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = 0; c < 6; ++c) m[r][c] = Hin[r * 6 + c];
    int tr[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int big = k;
        double bv = fabs(m[k][k]);
#pragma unroll
        for (int i = k + 1; i < 6; ++i) if (fabs(m[i][i]) > bv) { bv = fabs(m[i][i]); big = i; }
        tr[k] = big;
#pragma unroll
        for (int i = k + 1; i < 6; ++i) {
            if (big == i) {
#pragma unroll
                for (int j = 0; j < k; ++j) dswap(m[k][j], m[i][j]);
#pragma unroll
                for (int r = i + 1; r < 6; ++r) dswap(m[r][k], m[r][i]);
                dswap(m[k][k], m[i][i]);
#pragma unroll
                for (int r = k + 1; r < i; ++r) { const double t = m[r][k]; m[r][k] = m[i][r]; m[i][r] = t; }
            }
        }
        if (k > 0) {
            double temp[6];
#pragma unroll
            for (int j = 0; j < k; ++j) temp[j] = m[j][j] * m[k][j];
            double acc = 0.0;
#pragma unroll
            for (int j = 0; j < k; ++j) acc += m[k][j] * temp[j];
            m[k][k] -= acc;
#pragma unroll
            for (int i = k + 1; i < 6; ++i) {
                double a = 0.0;
#pragma unroll
                for (int j = 0; j < k; ++j) a += m[i][j] * temp[j];
                m[i][k] -= a;
            }
        }
        const double akk = m[k][k];
        const bool valid = fabs(akk) > 0.0;
        if (k == 0 && !valid) {
#pragma unroll
            for (int i = 0; i < 6; ++i) x[i] = 0.0;
            return;
        }
        if (valid) {
#pragma unroll
            for (int i = k + 1; i < 6; ++i) m[i][k] /= akk;
        }
    }
    double d[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) d[i] = b[i];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
#pragma unroll
        for (int i = k + 1; i < 6; ++i) if (tr[k] == i) dswap(d[k], d[i]);
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double a = 0.0;
#pragma unroll
        for (int j = 0; j < i; ++j) a += m[i][j] * d[j];
        d[i] -= a;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) d[i] = (fabs(m[i][i]) > DBL_MIN) ? d[i] / m[i][i] : 0.0;
#pragma unroll
    for (int i = 5; i >= 0; --i) {
        double a = 0.0;
#pragma unroll
        for (int j = i + 1; j < 6; ++j) a += m[j][i] * d[j];
        d[i] -= a;
    }
#pragma unroll
    for (int k = 5; k >= 0; --k) {
#pragma unroll
        for (int i = k + 1; i < 6; ++i) if (tr[k] == i) dswap(d[k], d[i]);
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = d[i];
}

// NT fixes the summation pattern of the nrows x kNE block partials (part_src: global or LDS) into tot[kNE] (LDS);
// the calling block may be larger than NT (its extra threads only join the barriers).
template <int NT, bool SC1 = false>
__device__ __forceinline__ void solve_sums(const double* part_src, int nrows, double* tot) {
    constexpr int kQ = NT / kNE;                     // partial rows per entry (36 for 1024 threads, 9 for 256)
    __shared__ double part[kQ][kNE];
    const int tid = threadIdx.x;
    if (tid < kQ * kNE) {
        // thread t sums flat entries t, t + kQ*kNE, ... of part_src[nrows][kNE]: coalesced, entry = t % kNE
        const int k = tid % kNE, q = tid / kNE;
        const double* src = part_src + tid;
        const int nrow = (nrows - q + kQ - 1) / kQ;
        constexpr size_t kStride = static_cast<size_t>(kQ) * kNE;
        double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};   // 8 independent loads in flight
        int j = 0;
        for (; j + 8 <= nrow; j += 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) a[u] += Mem<SC1>::ld(src + static_cast<size_t>(j + u) * kStride);
        }
        for (; j < nrow; ++j) a[0] += Mem<SC1>::ld(src + static_cast<size_t>(j) * kStride);
        part[q][k] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    }
    __syncthreads();
    if (tid < kNE) {
        double s = 0.0;
        for (int q = 0; q < kQ; ++q) s += part[q][tid];
        tot[tid] = s;
    }
    __syncthreads();
}

// One lane: H, g, cost from the summed normal equations, pivoted LDLT (:418), SE3 right-update of pose_old into
// pose_new with SO(3) re-projection (:422-434) and the convergence test (:437-448).  L (nullable) receives the
// iteration's log except n_corr / scale / alpha.  pose_old may alias pose_new's source state (read first).
__device__ inline bool solve_step(const KParams& P, const double* tot, const float* pose_old, float* pose_new,
                                  lo_iter_log* L) {
    double H[36], g[6];
    int k = 0;
    for (int r = 0; r < 6; ++r)
        for (int c = 0; c <= r; ++c) { H[r * 6 + c] = tot[k]; H[c * 6 + r] = tot[k]; ++k; }
    for (int j = 0; j < 6; ++j) g[j] = tot[21 + j];
    const double cost = tot[27];
    double mg[6], dd[6];
    for (int j = 0; j < 6; ++j) mg[j] = -g[j];
    ldlt6_solve(H, mg, dd);                                           // :418
    float delta[6];
    for (int j = 0; j < 6; ++j) delta[j] = static_cast<float>(dd[j]);
    const float dt[3] = {delta[0], delta[1], delta[2]}, dw[3] = {delta[3], delta[4], delta[5]};

    float R[9], t[3];
    for (int r = 0; r < 3; ++r) { for (int c = 0; c < 3; ++c) R[r * 3 + c] = pose_old[r * 4 + c]; t[r] = pose_old[r * 4 + 3]; }
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
    for (int r = 0; r < 3; ++r) { for (int c = 0; c < 3; ++c) pose_new[r * 4 + c] = Rn[r * 3 + c]; pose_new[r * 4 + 3] = tn[r]; }

    const float tdel = sqrtf(dot3f(dt[0], dt[1], dt[2], dt[0], dt[1], dt[2]));
    const float rdel = sqrtf(dot3f(dw[0], dw[1], dw[2], dw[0], dw[1], dw[2]));
    if (L) {
        for (int q = 0; q < 12; ++q) L->pose[q] = pose_new[q];
        L->cost = static_cast<float>(cost);
        k = 0;
        for (int r = 0; r < 6; ++r) for (int c = r; c < 6; ++c) L->H[k++] = static_cast<float>(H[r * 6 + c]);
        for (int j = 0; j < 6; ++j) { L->g[j] = static_cast<float>(g[j]); L->delta[j] = delta[j]; }
    }
    return tdel < P.tol_t && rdel < P.tol_r;                          // :443-448
}

// solve_step, and with publish also the GN state (pose, per-iteration log, iteration count, convergence flag).
// Returns the convergence test.  pose_old may alias DevState::pose (it is read before anything is written).
__device__ inline bool solve_core(const KParams& P, int it, const double* tot, const float* pose_old, float* pose_new,
                                  bool publish) {
    DevState* st = P.st;
    if (!publish) return solve_step(P, tot, pose_old, pose_new, nullptr);
    lo_iter_log Lg;
    const bool conv = solve_step(P, tot, pose_old, pose_new, &Lg);
    for (int q = 0; q < 12; ++q) st->pose[q] = pose_new[q];
    if (it < LO_MAX_ITERS) {                                          // the loop-closure ICP runs up to 100
        lo_iter_log& L = st->logs[it];
        L = Lg;
        L.n_corr = st->n_corr;
        L.scale = st->scale;
        L.alpha = st->alpha;
    }
    st->iter = it + 1;
    if (conv) st->done = 1;
    return conv;
}

// The selection of GN iteration it among the candidates the PKO launch already solved (P.cand_rec; pko_select_index:
// the reference's first strict JS minimum, AdaptiveMEstimator.cpp:256-275): the block's wave 0 loads the selected
// 48-word record into s_rec, block 0's thread 0 publishes it as the iteration's pose, log and convergence test
// (:417-448).  Returns false when the block has nothing to do (the scan already converged, or a tail launch whose
// scan is final); otherwise s_rec holds the record and *conv its convergence flag.  Every thread calls it (one
// barrier).  k_pick_correspond / k_pick (lo_kernels.hip) and k_pick_knn (lo_kdtree.hip).
__device__ __forceinline__ bool pick_select(const KParams& P, int it, float* s_rec, bool* conv) {
    DevState* st = P.st;
    const int tid = threadIdx.x;
    const int done = st->done || tail_gone(P);
    __shared__ int s_skip;
    __shared__ double s_alpha;
    if (tid < kWave) {
        const int bi = pko_select_index(P, P.js);
        const int c = bi > 0 ? bi - 1 : P.NA;
        if (tid < kCandWords) s_rec[tid] = P.cand_rec[static_cast<size_t>(c) * kCandWords + tid];
        if (tid == 0) {                           // thread 0's view of the flag decides for the whole block
            s_skip = done;
            s_alpha = bi > 0 ? P.alphas[bi] : P.min_scale;
        }
    }
    __syncthreads();
    if (s_skip) return false;
    *conv = s_rec[kCandConv] != 0.0f;
    if (blockIdx.x == 0 && tid == 0) {
        if (it < LO_MAX_ITERS) {                  // the loop-closure ICP runs up to 100
            lo_iter_log& L = st->logs[it];
#pragma unroll
            for (int q = 0; q < 12; ++q) L.pose[q] = s_rec[q];
            L.n_corr = st->n_corr;
            L.scale = st->scale;
            L.alpha = s_alpha;
            L.cost = s_rec[kCandCost];
#pragma unroll
            for (int q = 0; q < 21; ++q) L.H[q] = s_rec[kCandH + q];
#pragma unroll
            for (int q = 0; q < 6; ++q) { L.g[q] = s_rec[kCandG + q]; L.delta[q] = s_rec[kCandD + q]; }
        }
#pragma unroll
        for (int q = 0; q < 12; ++q) st->pose[q] = s_rec[q];
        st->alpha = s_alpha;
        st->iter = it + 1;
        if (*conv) st->done = 1;
        if (*conv || it + 1 >= P.max_iters) publish_final(P);   // the scan's result is final (scan pipeline)
    }
    return true;
}

}  // namespace lo
