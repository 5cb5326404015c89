// lo_exact.h — the reference's own fp32 operation order for one GN step (reference-exact mode, lo_set_exact):
// the per-correspondence Jacobian / weight / residual terms of build_ne (IterativeClosestPointOptimizer.cpp:345-410),
// Eigen's fp32 LDLT (:418) and the SO3::Exp / SO3(Matrix3f) re-projected right-update (:420-448, MathUtils.cpp:23-39,
// :86-99), restated as the oracle states them (oracle/src/lo_oracle.cpp build_ne / ldlt6_solve / so3_exp / se3_mul).
// Shared by the sequential-sum solve (lo_exact.hip k_exact_solve) and the speculative exact candidates of the PKO
// launch (lo_pko_body.h acc_candidate_exact).
#pragma once
#include <cfloat>

#include "lo_device.h"
#include "lo_math.h"

namespace lo {

constexpr int kExactTerms = 43;        // H (36, full: the reference's H is not symmetrised), g (6), cost
constexpr int kExactFactors = 14;      // per point: J (6), w J (6), w r, r (exact_point_factors)
#ifndef LO_EXACT_FACTORED
#define LO_EXACT_FACTORED 1
#endif
// long sums (term-major): k_exact_terms writes the 14 factor rows and the column sums form each term (1), or it writes
// the 43 term columns (0, A/B)
constexpr bool kExactFactored = LO_EXACT_FACTORED != 0;

// ---- the reference's fp32 solve and pose update (restated exactly as the oracle states them) ----
// LDLT<Matrix<float,6,6>> (Eigen ldlt_inplace<Lower>::unblocked with diagonal pivoting + LDLT::_solve_impl)
__device__ inline void ldlt6_solve_f32(const float (&Hin)[36], const float (&b)[6], float (&x)[6]) {
    float m[6][6];
#pragma unroll
    for (int r = 0; r < 6; ++r) for (int c = 0; c < 6; ++c) m[r][c] = Hin[r * 6 + c];
    int transp[6];
    float temp[6];
    bool zero_all = false;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int big = k;
        float bv = fabsf(m[k][k]);
#pragma unroll
        for (int i = k + 1; i < 6; ++i) if (fabsf(m[i][i]) > bv) { bv = fabsf(m[i][i]); big = i; }
        transp[k] = big;
        // the symmetric pivot swap with compile-time indices only (one unrolled candidate per row): a runtime index
        // into m would put the matrix in scratch memory
#pragma unroll
        for (int q = k + 1; q < 6; ++q) {
            if (q != big) continue;
#pragma unroll
            for (int j = 0; j < k; ++j) { const float t = m[k][j]; m[k][j] = m[q][j]; m[q][j] = t; }
#pragma unroll
            for (int i = q + 1; i < 6; ++i) { const float t = m[i][k]; m[i][k] = m[i][q]; m[i][q] = t; }
            { const float t = m[k][k]; m[k][k] = m[q][q]; m[q][q] = t; }
#pragma unroll
            for (int i = k + 1; i < q; ++i) { const float t = m[i][k]; m[i][k] = m[q][i]; m[q][i] = t; }
        }
        if (k > 0) {
#pragma unroll
            for (int j = 0; j < k; ++j) temp[j] = m[j][j] * m[k][j];
            float acc = 0.0f;
#pragma unroll
            for (int j = 0; j < k; ++j) acc += m[k][j] * temp[j];
            m[k][k] -= acc;
#pragma unroll
            for (int i = k + 1; i < 6; ++i) {
                float a = 0.0f;
#pragma unroll
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
#pragma unroll
    for (int i = 0; i < 6; ++i) d[i] = b[i];
#pragma unroll
    for (int k = 0; k < 6; ++k)
#pragma unroll
        for (int q = k + 1; q < 6; ++q) if (transp[k] == q) { const float t = d[k]; d[k] = d[q]; d[q] = t; }
#pragma unroll
    for (int i = 0; i < 6; ++i) { float a = 0.0f; for (int j = 0; j < i; ++j) a += m[i][j] * d[j]; d[i] -= a; }
#pragma unroll
    for (int i = 0; i < 6; ++i) d[i] = (fabsf(m[i][i]) > FLT_MIN) ? d[i] / m[i][i] : 0.0f;
#pragma unroll
    for (int i = 5; i >= 0; --i) { float a = 0.0f; for (int j = i + 1; j < 6; ++j) a += m[j][i] * d[j]; d[i] -= a; }
#pragma unroll
    for (int k = 5; k >= 0; --k)
#pragma unroll
        for (int q = k + 1; q < 6; ++q) if (transp[k] == q) { const float t = d[k]; d[k] = d[q]; d[q] = t; }
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = d[i];
}

__device__ inline float norm3e(const float* v) { return sqrtf(dot3e(v[0], v[1], v[2], v[0], v[1], v[2])); }

// SO3::Exp (MathUtils.cpp:23-39, kEps 1e-6f) with the SO3(Matrix3f) re-projection of its result; sin / cos are
// glibc's sinf / cosf restated (lo_math.h sincosf_ref: bit-identical to the reference's std::sin / std::cos of a
// float; r05 rounded the fp64 sin / cos instead, which differs from sinf in the last bit for 0.4 % of the floats in
// [1e-7, 0.8], and its device sin / cos took ~4.5k cycles of the solve's ~21k)
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
        const float s = sincosf_ref(theta, 0);
        const float omc = 1.0f - sincosf_ref(theta, 1);
        float sK[3][3], KK[3][3];
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) sK[r][c] = omc * K[r][c];
        mul33e(sK, K, KK);
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) M[r][c] = ((r == c ? 1.0f : 0.0f) + s * K[r][c]) + KK[r][c];
    }
    so3_project_svd(M, R);
}

// One correspondence's factors of the 43 terms (:364-404): J (6), w J (6), w r, r -- the terms themselves are
// H[row][col] = J[col] * (w J[row]), g[j] = (w r) * J[j], cost = (w r) * r, each one fp32 product.
__device__ __forceinline__ void exact_point_factors(const KParams& P, const float (&T)[12], double scale, float dl,
                                                    double r64, float px, float py, float pz, const Slot& sl,
                                                    float (&f)[14]) {
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
#pragma unroll
    for (int j = 0; j < 6; ++j) { f[j] = J[j]; f[6 + j] = w * J[j]; }
    f[12] = w * res;
    f[13] = res;
}
// Term k of the 43 (row-major H, then g, then cost) as the product of factors fa[k] * fb[k].
__device__ __forceinline__ void exact_term_factors(int k, int& fa, int& fb) {
    if (k < 36) { fa = k % 6; fb = 6 + k / 6; }          // J[col] * wJ[row]
    else if (k < 42) { fa = 12; fb = k - 36; }           // wr * J[j]
    else { fa = 12; fb = 13; }                           // wr * r
}

// The reference's solve and right-update from the 43 sums (:417-448): pn = the new pose, delta, convergence.
__device__ inline bool exact_solve_step(const float (&tot)[kExactTerms], const float pose[12], double tol_t, double tol_r,
                                        float (&pn)[12], float (&delta)[6]) {
    float Hf[36], mg[6];
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
    for (int r = 0; r < 3; ++r) { for (int c = 0; c < 3; ++c) R[r][c] = pose[r * 4 + c]; t[r] = pose[r * 4 + 3]; }
    mul33e(R, Rd, M);                                           // SE3::operator* (MathUtils.h:144-147)
    so3_project_svd(M, Rn);
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) pn[r * 4 + c] = Rn[r][c];
        pn[r * 4 + 3] = t[r] + dot3e(R[r][0], R[r][1], R[r][2], dt[0], dt[1], dt[2]);
    }
    return norm3e(dt) < tol_t && norm3e(dw) < tol_r;          // :443-448
}

}  // namespace lo
