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
#include <cfloat>

#include "lo_device.h"
#include "lo_math.h"

namespace lo {

constexpr int kExactTerms = 43;        // H (36, full: the reference's H is not symmetrised), g (6), cost

// ---- the reference's fp32 solve and pose update (restated exactly as the oracle states them) ----
// LDLT<Matrix<float,6,6>> (Eigen ldlt_inplace<Lower>::unblocked with diagonal pivoting + LDLT::_solve_impl)
__device__ inline void ldlt6_solve_f32(const float (&Hin)[36], const float (&b)[6], float (&x)[6]) {
    float m[6][6];
    for (int r = 0; r < 6; ++r) for (int c = 0; c < 6; ++c) m[r][c] = Hin[r * 6 + c];
    int transp[6];
    float temp[6];
    bool zero_all = false;
    for (int k = 0; k < 6; ++k) {
        int big = k;
        float bv = fabsf(m[k][k]);
        for (int i = k + 1; i < 6; ++i) if (fabsf(m[i][i]) > bv) { bv = fabsf(m[i][i]); big = i; }
        transp[k] = big;
        if (k != big) {
            for (int j = 0; j < k; ++j) { const float t = m[k][j]; m[k][j] = m[big][j]; m[big][j] = t; }
            for (int i = big + 1; i < 6; ++i) { const float t = m[i][k]; m[i][k] = m[i][big]; m[i][big] = t; }
            { const float t = m[k][k]; m[k][k] = m[big][big]; m[big][big] = t; }
            for (int i = k + 1; i < big; ++i) { const float t = m[i][k]; m[i][k] = m[big][i]; m[big][i] = t; }
        }
        if (k > 0) {
            for (int j = 0; j < k; ++j) temp[j] = m[j][j] * m[k][j];
            float acc = 0.0f;
            for (int j = 0; j < k; ++j) acc += m[k][j] * temp[j];
            m[k][k] -= acc;
            for (int i = k + 1; i < 6; ++i) {
                float a = 0.0f;
                for (int j = 0; j < k; ++j) a += m[i][j] * temp[j];
                m[i][k] -= a;
            }
        }
        const float akk = m[k][k];
        const bool valid = fabsf(akk) > 0.0f;
        if (k == 0 && !valid) { zero_all = true; break; }
        if (k < 5 && valid) for (int i = k + 1; i < 6; ++i) m[i][k] /= akk;
    }
    if (zero_all) { for (int i = 0; i < 6; ++i) x[i] = 0.0f; return; }
    float d[6];
    for (int i = 0; i < 6; ++i) d[i] = b[i];
    for (int k = 0; k < 6; ++k) if (transp[k] != k) { const float t = d[k]; d[k] = d[transp[k]]; d[transp[k]] = t; }
    for (int i = 0; i < 6; ++i) { float a = 0.0f; for (int j = 0; j < i; ++j) a += m[i][j] * d[j]; d[i] -= a; }
    for (int i = 0; i < 6; ++i) d[i] = (fabsf(m[i][i]) > FLT_MIN) ? d[i] / m[i][i] : 0.0f;
    for (int i = 5; i >= 0; --i) { float a = 0.0f; for (int j = i + 1; j < 6; ++j) a += m[j][i] * d[j]; d[i] -= a; }
    for (int k = 5; k >= 0; --k) if (transp[k] != k) { const float t = d[k]; d[k] = d[transp[k]]; d[transp[k]] = t; }
    for (int i = 0; i < 6; ++i) x[i] = d[i];
}

__device__ inline float norm3e(const float* v) { return sqrtf(dot3e(v[0], v[1], v[2], v[0], v[1], v[2])); }

// SO3::Exp (MathUtils.cpp:23-39, kEps 1e-6f) with the SO3(Matrix3f) re-projection of its result; sin / cos are
// evaluated in fp64 and rounded (the correctly rounded fp32 value; glibc's sinf agrees with it for 99.6 % of the
// floats in [1e-7, 0.8], cosf for 99.99 %)
__device__ inline void so3_exp_exact(const float w[3], float R[3][3]) {
    const float theta = norm3e(w);
    float M[3][3];
    if (theta < 1e-6f) {
        const float H[3][3] = {{0.0f, -w[2], w[1]}, {w[2], 0.0f, -w[0]}, {-w[1], w[0], 0.0f}};
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) M[r][c] = (r == c ? 1.0f : 0.0f) + H[r][c];
    } else {
        const float ti = 1.0f / theta;
        const float k[3] = {w[0] * ti, w[1] * ti, w[2] * ti};
        const float K[3][3] = {{0.0f, -k[2], k[1]}, {k[2], 0.0f, -k[0]}, {-k[1], k[0], 0.0f}};
        const float s = static_cast<float>(sin(static_cast<double>(theta)));
        const float omc = 1.0f - static_cast<float>(cos(static_cast<double>(theta)));
        float sK[3][3], KK[3][3];
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) sK[r][c] = omc * K[r][c];
        mul33e(sK, K, KK);
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) M[r][c] = ((r == c ? 1.0f : 0.0f) + s * K[r][c]) + KK[r][c];
    }
    so3_project_svd(M, R);
}

// ---- iteration 0: scale = sqrt(var) / 6 of the residuals sorted ascending, mean and variance summed in that order
// (IterativeClosestPointOptimizer.cpp:304-316).  One workgroup: the residuals of the accepted points (+inf for the
// rest) in dynamic LDS, bitonic sort, then one lane accumulates as std::accumulate does ----
constexpr int kExactScaleThreads = 1024;

// acc += v_0 + v_1 + ... + v_{cnt-1}, one rounding per element in index order (v_k = x_k, or (x_k - m)^2 with SQ), as
// one wave-uniform chain: each 16-lane row holds 16 consecutive elements in a register and v_fmac_f64_dpp with a
// row_newbcast source adds element 16c + N as acc = fma(v, 1.0, acc), which rounds exactly as acc + v -- no LDS
// round trip between the adds (one lane reading LDS per element was ~25x slower).  Wave 0 only; elements past cnt
// are never broadcast (the row guard) and never read.
template <int N>
__device__ __forceinline__ void bcast_add(double& acc, double v, double one) {
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(v), "v"(one), "i"(N));
}
template <int N>
__device__ __forceinline__ void bcast_add_row(double& acc, double v, double one, int left) {
    if constexpr (N < 16) {
        if (N < left) {
            bcast_add<N>(acc, v, one);
            bcast_add_row<N + 1>(acc, v, one, left);
        }
    }
}
template <bool SQ>
__device__ __forceinline__ void seq_sum_rows(const double* s_x, int cnt, double m, double& acc) {
    constexpr int kW = 4;                                  // rows of 16 elements per window
    const int n16 = threadIdx.x & 15;
    const double one = 1.0;
    double cur[kW], nxt[kW];
#pragma unroll
    for (int w = 0; w < kW; ++w) cur[w] = (16 * w + n16 < cnt) ? s_x[16 * w + n16] : 0.0;
    for (int base = 0; base < cnt; base += 16 * kW) {
#pragma unroll
        for (int w = 0; w < kW; ++w) {
            const int i = base + 16 * (kW + w) + n16;
            nxt[w] = (i < cnt) ? s_x[i] : 0.0;
        }
        double v[kW];
#pragma unroll
        for (int w = 0; w < kW; ++w) {
            if constexpr (SQ) { const double d = cur[w] - m; v[w] = d * d; } else { v[w] = cur[w]; }
        }
        // the DPP sources above were written by VALU ops: two wait states before the first broadcast read
        asm volatile("s_nop 1" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
#pragma unroll
        for (int w = 0; w < kW; ++w) bcast_add_row<0>(acc, v[w], one, cnt - (base + 16 * w));
#pragma unroll
        for (int w = 0; w < kW; ++w) cur[w] = nxt[w];
    }
}
__global__ __launch_bounds__(kExactScaleThreads) void k_exact_scale(KParams P, int n2) {
    DevState* st = P.st;
    if (st->done) return;
    extern __shared__ double s_r[];
    const int tid = threadIdx.x, n = scan_n(P);
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
    for (int i = tid; i < n2; i += kExactScaleThreads) {
        double v = __builtin_inf();
        if (i < n) {
            const int s = P.slot[i];
            if (s >= 0 && P.kd_res) {
                v = P.kd_res[i];                           // KDTree variant: the plane distance it accepted
            } else if (s >= 0) {
                float wx, wy, wz;
                transform_pt(T, P.pts[3 * i], P.pts[3 * i + 1], P.pts[3 * i + 2], wx, wy, wz);
                v = residual_f64(P.tab[s], wx, wy, wz);
            }
        }
        s_r[i] = v;
    }
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < n2; i += kExactScaleThreads) {
                const int l = i ^ j;
                if (l > i) {
                    const double a = s_r[i], b = s_r[l];
                    const bool up = (i & k) == 0;
                    if (up ? (a > b) : (a < b)) { s_r[i] = b; s_r[l] = a; }
                }
            }
            __syncthreads();
        }
    }
    // cnt = the first +inf (the unaccepted points sort last), found in parallel
    __shared__ int s_cnt;
    if (tid == 0) s_cnt = n;
    __syncthreads();
    for (int i = tid; i < n; i += kExactScaleThreads)
        if (s_r[i] == __builtin_inf() && (i == 0 || s_r[i - 1] != __builtin_inf())) atomicMin(&s_cnt, i);
    __syncthreads();
    if (tid >= kWave) return;
    const int cnt = s_cnt;
    if (cnt == 0) return;                                  // too few correspondences: the PKO launch reports it
    // std::accumulate in sorted order, then the variance loop, each one sequential chain run by wave 0
    double sum = 0.0;
    seq_sum_rows<false>(s_r, cnt, 0.0, sum);
    const double mean = sum / cnt;
    double var = 0.0;
    seq_sum_rows<true>(s_r, cnt, mean, var);
    var /= cnt;
    if (tid == 0) st->scale = sqrt(var) / 6.0;
}

// ---- iteration 0 for scans beyond the one-workgroup sort (kExactMaxPoints < n): k_exact_resid writes every point's
// residual (+inf without a correspondence) to global memory, the context sorts them ascending (hipCUB radix sort:
// the same order as std::sort for the non-NaN values; -0 / +0 ties do not change any sum), and k_exact_scale_g
// finds the first +inf and runs the two sequential sums over the sorted residuals, staged through LDS by the
// copy waves as in k_exact_solve ----
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

constexpr int kScaleGThreads = 1024;
constexpr int kScaleGChunk = 4096;                             // doubles per staged chunk (2 x 32 KB of LDS)
template <bool SQ>
__device__ __forceinline__ void staged_seq_sum(const double* __restrict__ x, int cnt, double m, double& acc,
                                               double (*buf)[kScaleGChunk]) {
    const int tid = threadIdx.x;
    const int n_chunks = (cnt + kScaleGChunk - 1) / kScaleGChunk;
    for (int k = tid; k < kScaleGChunk && k < cnt; k += kScaleGThreads) buf[0][k] = x[k];
    __syncthreads();
    for (int c = 0; c < n_chunks; ++c) {
        if (tid >= kWave) {                                    // copy chunk c + 1
            const int base = (c + 1) * kScaleGChunk;
            for (int k = tid - kWave; k < kScaleGChunk && base + k < cnt; k += kScaleGThreads - kWave)
                buf[(c + 1) & 1][k] = x[base + k];
        } else {
            seq_sum_rows<SQ>(buf[c & 1], min(kScaleGChunk, cnt - c * kScaleGChunk), m, acc);
        }
        __syncthreads();
    }
}
__global__ __launch_bounds__(kScaleGThreads) void k_exact_scale_g(KParams P, const double* __restrict__ sorted) {
    DevState* st = P.st;
    if (st->done) return;
    __shared__ double buf[2][kScaleGChunk];
    __shared__ int s_cnt;
    const int tid = threadIdx.x, n = scan_n(P);
    if (tid == 0) s_cnt = n;
    __syncthreads();
    for (int i = tid; i < n; i += kScaleGThreads)
        if (sorted[i] == __builtin_inf() && (i == 0 || sorted[i - 1] != __builtin_inf())) atomicMin(&s_cnt, i);
    __syncthreads();
    const int cnt = s_cnt;
    if (cnt == 0) return;                                      // too few correspondences: the PKO launch reports it
    double sum = 0.0;
    staged_seq_sum<false>(sorted, cnt, 0.0, sum, buf);
    // wave 0 holds the sum; the mean goes to every wave through LDS (the other waves keep copying)
    __shared__ double s_mean;
    if (tid == 0) s_mean = sum / cnt;
    __syncthreads();
    const double mean = s_mean;
    double var = 0.0;
    staged_seq_sum<true>(sorted, cnt, mean, var, buf);
    if (tid == 0) st->scale = sqrt(var / cnt) / 6.0;
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
    float* out = P.ex_terms + static_cast<size_t>(i) * kExactTerms;
    const int s = P.slot[i];
    if (s < 0) {
        for (int k = 0; k < kExactTerms; ++k) out[k] = 0.0f;
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
    const float nres = static_cast<float>(r64 / std_max(scale, 1e-6));
    const float qx = dot3f(T[0], T[1], T[2], px, py, pz) + T[3];
    const float qy = dot3f(T[4], T[5], T[6], px, py, pz) + T[7];
    const float qz = dot3f(T[8], T[9], T[10], px, py, pz) + T[11];
    const float n0 = sl.n[0], n1 = sl.n[1], n2 = sl.n[2];
    const float res = dot3f(n0, n1, n2, qx - sl.c[0], qy - sl.c[1], qz - sl.c[2]);
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
    if (P.robust) {
        const float an = fabsf(nres);
        if (P.cauchy_loss) { const float ratio = an / dl; w = 1.0f / (1.0f + ratio * ratio); }
        else if (an > dl) w = dl / an;
    }
    float wJ[6];
    for (int j = 0; j < 6; ++j) wJ[j] = w * J[j];
    for (int row = 0; row < 6; ++row)
        for (int col = 0; col < 6; ++col) out[row * 6 + col] = J[col] * wJ[row];
    const float wr = w * res;
    for (int j = 0; j < 6; ++j) out[36 + j] = wr * J[j];
    out[42] = wr * res;
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
    float Hf[36], mg[6], delta[6];
    for (int k = 0; k < 36; ++k) Hf[k] = tot[k];
    for (int j = 0; j < 6; ++j) mg[j] = -tot[36 + j];
    ldlt6_solve_f32(Hf, mg, delta);                            // :418
    const float dt[3] = {delta[0], delta[1], delta[2]}, dw[3] = {delta[3], delta[4], delta[5]};
    float Rd[3][3];
    if (norm3e(dw) < 1e-10f) {                                 // :427-431
        const float I[3][3] = {{1.0f, 0.0f, 0.0f}, {0.0f, 1.0f, 0.0f}, {0.0f, 0.0f, 1.0f}};
        so3_project_svd(I, Rd);
    } else {
        so3_exp_exact(dw, Rd);
    }
    float R[3][3], t[3], M[3][3], Rn[3][3];
    for (int r = 0; r < 3; ++r) { for (int c = 0; c < 3; ++c) R[r][c] = st->pose[r * 4 + c]; t[r] = st->pose[r * 4 + 3]; }
    mul33e(R, Rd, M);                                           // SE3::operator* (MathUtils.h:144-147)
    so3_project_svd(M, Rn);
    float pn[12];
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) pn[r * 4 + c] = Rn[r][c];
        pn[r * 4 + 3] = t[r] + dot3e(R[r][0], R[r][1], R[r][2], dt[0], dt[1], dt[2]);
    }
    const bool conv = norm3e(dt) < P.tol_t && norm3e(dw) < P.tol_r;   // :443-448
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
