// lo_kernels.hip — HIP kernels of the point-to-plane ICP hot path for gfx950 (MI355X / CDNA4).
//
// One Gauss-Newton iteration of IterativeClosestPointOptimizer::optimize
// (reference src/optimization/IterativeClosestPointOptimizer.cpp:281-449) is four launches on one stream:
//   k_correspond  per point: transform, L1 surfel probe, fp64 residual, accept r <= max_corr
//                 (find_correspondences :587-645); per-wave validity ballots; iteration 0 also the
//                 per-block residual sum / M2 for the normalisation scale (:304-316)
//   k_pko         (lo_pko.hip) correspondence count, scale, the reference's PKO sample selection, GMM fit
//                 and the JS-divergence alpha grid (AdaptiveMEstimator.cpp:243-485, :710-787)
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
// init: first launch of a scan.  The GN state reset (k_init's job) is folded in here -- the pose comes from
// the kernel argument (T0 / T0p), block 0 writes the fresh DevState that the later kernels of the scan read.
// The point load is issued before the DevState loads (done flag, pose) so the three latencies overlap
// instead of serialising at the start of every wave.
__device__ __forceinline__ void correspond_tail(const KParams& P, const float (&T)[12], float px, float py, float pz,
                                                int i, int n, int with_stats, int blk) {
    int slot = -1;
    double r = 0.0;
    if (i < n) {
        float wx, wy, wz;
        transform_pt(T, px, py, pz, wx, wy, wz);
        const int s = lookup_surfel(P.tab, P.log2cap, P.l1scale, wx, wy, wz);
        if (s >= 0) {
            r = residual_f64(P.tab[s], wx, wy, wz);
            if (!(r > P.maxd)) slot = s;     // reference rejects only residual > max (NaN kept, :630)
        }
        P.slot[i] = slot;
        if (P.res_dbg) P.res_dbg[i] = slot >= 0 ? r : 0.0;
    }
    corr_epilogue(P, slot >= 0, r, with_stats, blk);
}

__device__ __forceinline__ void correspond_body(const KParams& P, int with_stats, int init, int blk) {
    const int i = blk * kBlock + threadIdx.x;
    const int n = scan_n(P);
    float px = 0.0f, py = 0.0f, pz = 0.0f;
    if (i < n) { px = P.pts[3 * i]; py = P.pts[3 * i + 1]; pz = P.pts[3 * i + 2]; }
    const DevState* cst = P.st;
    const int done = cst->done;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = cst->pose[k];
    if (!init && done) return;
    scan_pose(P, init, blk, T);
    correspond_tail(P, T, px, py, pz, i, n, with_stats, blk);
}

__global__ __launch_bounds__(kBlock) void k_correspond(KParams P, int with_stats) {
    correspond_body(P, with_stats, P.init, blockIdx.x);
}

// Batched launch (lo_batch_*): blockIdx.y = job (one context each: own scan, map and GN state); the grid is
// sized for the largest job and a job's surplus blocks leave before touching any of its buffers.
__global__ __launch_bounds__(kBlock) void k_correspond_b(const KParams* __restrict__ PB, int with_stats, int init) {
    const KParams& P = PB[blockIdx.y];
    if (static_cast<int>(blockIdx.x) >= P.nb) return;
    correspond_body(P, with_stats, init, blockIdx.x);
}

// ====================================================================================================
// k_accumulate
// ====================================================================================================
template <int NT>
__device__ void solve_tail(const KParams& P, int it, int ne_only, const double* part_src, int nrows);

// fuse: 0 = partials only, 1 = the last block to finish also runs the GN solve / update (k_solve's job),
// 2 = the last block writes the summed normal equations (lo_build_normal_equations)
__device__ __forceinline__ void accumulate_body(const KParams& P, int it, int fuse, int blk, int nblk) {
    DevState* st = P.st;
    if (st->done) return;
    __shared__ float s_acc[kWavesPerBlock][kNE];
    __shared__ double s_alpha;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // Huber delta of this iteration: argmin of the JS grid k_pko wrote (PKO), else robust_loss_delta
    if (wid == 0) {
        const double a = P.alpha_given ? P.st->alpha : (P.use_pko ? pko_select_alpha(P) : P.robust_delta);
        if (lane == 0) {
            s_alpha = a;
            if (blk == 0 && !P.alpha_given) P.st->alpha = a;
        }
    }
    __syncthreads();
    float acc[kNE];
#pragma unroll
    for (int k = 0; k < kNE; ++k) acc[k] = 0.0f;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
    const double scale = st->scale;
    const float dl = static_cast<float>(s_alpha);
    // grid-stride (at most kAccBlocks blocks): per-thread fp32 sums of <= 4 points at 1M, then the same
    // wave / block trees; the partial count k_solve reduces stays <= kAccBlocks
    const int n = scan_n(P);
    for (int i = blk * kBlock + tid; i < n; i += P.nb_acc * kBlock) acc_point(P, T, scale, dl, i, acc);
#pragma unroll
    for (int k = 0; k < kNE; ++k) {
        const float v = wave_total(acc[k]);
        if (lane == 0) s_acc[wid][k] = v;
    }
    __syncthreads();
    if (tid < kNE) {
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < kWavesPerBlock; ++w) v += static_cast<double>(s_acc[w][tid]);
        P.blk_part[static_cast<size_t>(blk) * kNE + tid] = v;
    }
    if (fuse == 0) return;
    // last-block-done: release the partials at agent scope (the 8 XCDs have separate L2s), count arrivals;
    // the block that arrives last acquires and reduces them in fixed block order -- one launch fewer per
    // GN iteration, same deterministic sum as a separate k_solve
    __shared__ int s_last;
    __threadfence();
    __syncthreads();
    if (tid == 0) s_last = (atomicAdd(&st->acc_arrive, 1u) == static_cast<unsigned>(nblk - 1)) ? 1 : 0;
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    if (tid == 0) st->acc_arrive = 0;
    solve_tail<kBlock>(P, it, fuse == 2, P.blk_part, P.nb_acc);
}

__global__ __launch_bounds__(kBlock) void k_accumulate(KParams P, int it, int fuse) {
    accumulate_body(P, it, fuse, blockIdx.x, gridDim.x);
}

// Batched launch for batches with a large job (> kFuseMaxBlocks blocks): blockIdx.y = job, partials only;
// k_solve_b reduces and solves every job.
__global__ __launch_bounds__(kBlock) void k_accumulate_b(const KParams* __restrict__ PB, int it) {
    const KParams& P = PB[blockIdx.y];
    if (static_cast<int>(blockIdx.x) >= P.nb_acc) return;
    accumulate_body(P, it, 0, blockIdx.x, P.nb_acc);
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
__device__ void so3_exp(const float* w, float* R) {
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

__device__ void ldlt6_solve(const double* Hin, const double* b, double* x) {
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
template <int NT>
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
            for (int u = 0; u < 8; ++u) a[u] += src[static_cast<size_t>(j + u) * kStride];
        }
        for (; j < nrow; ++j) a[0] += src[static_cast<size_t>(j) * kStride];
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
// pose_new with SO(3) re-projection (:422-434); with publish also the GN state (pose, per-iteration log, iteration
// count, convergence flag :437-448).  Returns the convergence test.  pose_old may alias DevState::pose (it is read
// before anything is written).
__device__ bool solve_core(const KParams& P, int it, const double* tot, const float* pose_old, float* pose_new,
                           bool publish) {
    DevState* st = P.st;
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
    const bool conv = tdel < P.tol_t && rdel < P.tol_r;               // :443-448
    if (!publish) return conv;
    for (int q = 0; q < 12; ++q) st->pose[q] = pose_new[q];
    if (it < LO_MAX_ITERS) {                                          // the loop-closure ICP runs up to 100
        lo_iter_log& L = st->logs[it];
        for (int q = 0; q < 12; ++q) L.pose[q] = pose_new[q];
        L.n_corr = st->n_corr;
        L.scale = st->scale;
        L.alpha = st->alpha;
        L.cost = static_cast<float>(cost);
        k = 0;
        for (int r = 0; r < 6; ++r) for (int c = r; c < 6; ++c) L.H[k++] = static_cast<float>(H[r * 6 + c]);
        for (int j = 0; j < 6; ++j) { L.g[j] = static_cast<float>(g[j]); L.delta[j] = delta[j]; }
    }
    st->iter = it + 1;
    if (conv) st->done = 1;
    return conv;
}

template <int NT>
__device__ void solve_tail(const KParams& P, int it, int ne_only, const double* part_src, int nrows) {
    DevState* st = P.st;
    __shared__ double tot[kNE];
    solve_sums<NT>(part_src, nrows, tot);
    if (threadIdx.x != 0) return;
    if (ne_only) {
        int k = 0;
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c <= r; ++c) { st->H_out[r * 6 + c] = tot[k]; st->H_out[c * 6 + r] = tot[k]; ++k; }
        for (int j = 0; j < 6; ++j) st->g_out[j] = tot[21 + j];
        st->cost_out = tot[27];
        return;
    }
    float pn[12];
    solve_core(P, it, tot, st->pose, pn, true);
}

// Standalone solve over all block partials (lo_bench_kernel; the GN loop fuses it into k_accumulate)
__global__ __launch_bounds__(kSolveThreads) void k_solve(KParams P, int it, int ne_only) {
    if (P.st->done) return;
    solve_tail<kSolveThreads>(P, it, ne_only, P.blk_part, P.nb_acc);
}

// Solve from the speculative normal equations (single scans with nb_acc <= kFuseMaxBlocks): the candidate of
// the selected alpha (acc_candidate, lo_pko.hip) holds the same per-block partials the fused k_accumulate would
// have formed, reduced here with the same solve_tail<kBlock> pattern -- bit-identical, one launch fewer.
__global__ __launch_bounds__(kBlock) void k_solve_pick(KParams P, int it) {
    DevState* st = P.st;
    if (st->done) return;
    __shared__ int s_c;
    if (threadIdx.x < kWave) {
        const int bi = pko_select_index(P);
        if (threadIdx.x == 0) {
            s_c = bi > 0 ? bi - 1 : P.NA;
            st->alpha = bi > 0 ? P.alphas[bi] : P.min_scale;
        }
    }
    __syncthreads();
    solve_tail<kBlock>(P, it, 0, P.acc_part + static_cast<size_t>(s_c) * kFuseMaxBlocks * kNE, P.nb_acc);
}

// The solve of GN iteration it fused with the correspondence search of iteration it + 1 (single small scans with
// PKO, surfel path): every block reduces the selected candidate's partials and solves redundantly -- same data,
// same code, so the same pose in every block -- then searches its 256 points with the new pose; block 0
// publishes the GN state.  The old pose is read from the previous iteration's log (the initial pose for it = 0),
// which no block of this launch writes.  One launch per GN iteration fewer than k_solve_pick + k_correspond.
__global__ __launch_bounds__(kBlock) void k_solve_correspond(KParams P, int it) {
    DevState* st = P.st;
    const int tid = threadIdx.x, blk = blockIdx.x;
    const int i = blk * kBlock + tid;
    const int n = scan_n(P);
    float px = 0.0f, py = 0.0f, pz = 0.0f;
    if (i < n) { px = P.pts[3 * i]; py = P.pts[3 * i + 1]; pz = P.pts[3 * i + 2]; }
    if (st->done) return;
    __shared__ int s_c, s_done;
    __shared__ double tot[kNE];
    __shared__ float s_T[12];
    if (tid < kWave) {
        const int bi = pko_select_index(P);
        if (tid == 0) {
            s_c = bi > 0 ? bi - 1 : P.NA;
            if (blk == 0) st->alpha = bi > 0 ? P.alphas[bi] : P.min_scale;
        }
    }
    __syncthreads();
    solve_sums<kBlock>(P.acc_part + static_cast<size_t>(s_c) * kFuseMaxBlocks * kNE, P.nb_acc, tot);
    if (tid == 0) {
        const float* pose_old = it == 0 ? P.T0 : st->logs[it - 1].pose;
        s_done = solve_core(P, it, tot, pose_old, s_T, blk == 0) ? 1 : 0;
    }
    __syncthreads();
    if (s_done) return;                          // converged: the later launches of the scan see DevState::done
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = s_T[k];
    correspond_tail(P, T, px, py, pz, i, n, 0, blk);
}

// Batched solve (jobs with more than kFuseMaxBlocks accumulate blocks present): one block per job, with the
// partial-sum pattern the single-scan path uses for that job's size, so every job stays bit-identical to it.
__global__ __launch_bounds__(kSolveThreads) void k_solve_b(const KParams* __restrict__ PB, int it) {
    const KParams& P = PB[blockIdx.x];
    if (P.st->done) return;
    if (P.nb_acc <= kFuseMaxBlocks) solve_tail<kBlock>(P, it, 0, P.blk_part, P.nb_acc);
    else solve_tail<kSolveThreads>(P, it, 0, P.blk_part, P.nb_acc);
}

// Batched accumulate + solve for small jobs (nb_acc <= kFuseMaxBlocks): ONE workgroup of 8 waves per job walks
// the job's 256-point blocks two at a time (wave w takes block 2r + w/4, its quarter w%4), so each point, wave
// sum and per-block fp64 partial is formed exactly as in the multi-block launch; the partials stay in LDS and the
// same workgroup solves.  No inter-workgroup hand-off: no atomics and no agent-scope fences (whose L2 write-back
// and invalidate per workgroup dominated the multi-block form once thousands of workgroups were in flight).
constexpr int kAcc1Threads = 512;
__global__ __launch_bounds__(kAcc1Threads) void k_accumulate_b1(const KParams* __restrict__ PB, int it) {
    const KParams& P = PB[blockIdx.y];
    DevState* st = P.st;
    if (st->done) return;
    constexpr int kW = kAcc1Threads / kWave;           // 8 waves = 2 virtual blocks per pass
    __shared__ float s_acc[kW][kNE];
    __shared__ double s_part[kFuseMaxBlocks * kNE];
    __shared__ double s_alpha;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (wid == 0) {
        const double a = P.use_pko ? pko_select_alpha(P) : P.robust_delta;
        if (lane == 0) { s_alpha = a; st->alpha = a; }
    }
    __syncthreads();
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
    const double scale = st->scale;
    const float dl = static_cast<float>(s_alpha);
    const int n = scan_n(P), nb = P.nb_acc;
    for (int vb0 = 0; vb0 < nb; vb0 += kW / kWavesPerBlock) {
        const int vb = vb0 + wid / kWavesPerBlock;
        const int i = vb * kBlock + (wid % kWavesPerBlock) * kWave + lane;
        float acc[kNE];
#pragma unroll
        for (int k = 0; k < kNE; ++k) acc[k] = 0.0f;
        if (vb < nb && i < n) acc_point(P, T, scale, dl, i, acc);
#pragma unroll
        for (int k = 0; k < kNE; ++k) {
            const float v = wave_total(acc[k]);
            if (lane == 0) s_acc[wid][k] = v;
        }
        __syncthreads();
        if (tid < kW / kWavesPerBlock * kNE) {
            const int q = tid / kNE, k = tid - q * kNE;
            if (vb0 + q < nb) {
                double v = 0.0;
#pragma unroll
                for (int w = 0; w < kWavesPerBlock; ++w) v += static_cast<double>(s_acc[q * kWavesPerBlock + w][k]);
                s_part[(vb0 + q) * kNE + k] = v;
            }
        }
        __syncthreads();
    }
    solve_tail<kBlock>(P, it, 0, s_part, nb);
}

// ====================================================================================================
// k_init: reset the GN state for a new scan.  The initial pose travels as a kernel argument, so any
// number of scans can be enqueued back to back without a host staging buffer.
// ====================================================================================================
struct Pose12 { float v[12]; };

__global__ void k_init(DevState* st, Pose12 T, double scale, double alpha) {
    if (threadIdx.x < 12) st->pose[threadIdx.x] = T.v[threadIdx.x];
    if (threadIdx.x == 0) {
        st->scale = scale;
        st->alpha = alpha;
        st->n_corr = 0;
        st->iter = 0;
        st->done = 0;
        st->status = LO_OK;
        st->acc_arrive = 0;
        st->kd_unres_n = 0;
        st->inliers = 0;
    }
}

// Copy the current pose + status into a caller buffer (16 floats: pose[12], status, iterations, n_corr, 0).
__global__ void k_export_pose(const DevState* st, float* out) {
    const int t = threadIdx.x;
    if (t < 12) out[t] = st->pose[t];
    if (t == 12) out[12] = static_cast<float>(st->status);
    if (t == 13) out[13] = static_cast<float>(st->iter);
    if (t == 14) out[14] = static_cast<float>(st->n_corr);
    if (t == 15) out[15] = 0.0f;
}

// Batched result export: one record per job (lo_batch_result reads them with one copy).
__global__ void k_export_batch(const KParams* __restrict__ PB, lo_batch_rec* out) {
    const DevState* st = PB[blockIdx.x].st;
    lo_batch_rec& R = out[blockIdx.x];
    const int t = threadIdx.x;
    if (t < 12) R.pose[t] = st->pose[t];
    if (t == 12) R.status = st->status;
    if (t == 13) R.iterations = st->iter;
    if (t == 14) R.n_corr = st->n_corr;
    if (t == 15) R.alpha = st->alpha;
    if (t == 16) R.initial_cost = st->iter > 0 ? st->logs[0].cost : 0.0f;
    if (t == 17) R.final_cost = st->iter > 0 ? st->logs[min(st->iter, LO_MAX_ITERS) - 1].cost : 0.0f;
}

}  // namespace lo

