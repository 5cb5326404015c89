// lo_math.h — host-side fp32 restatements of the reference's Eigen / MathUtils operations (shared by the
// host VoxelMap and the odometry loop).  Compiled with -ffp-contract=off: no FMA contraction where Eigen
// (GCC, no -mfma) rounds every product and sum separately.
#pragma once
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>

// The SVD / SO(3) restatements below also run on the device (lo_exact.hip): host-device under HIP.
#if defined(__HIP__)
#define LO_HD __host__ __device__
#else
#define LO_HD
#endif

namespace lo {

// ---------------------------------------------------------------------------------------------
// log(x) for the PKO JS terms (AdaptiveMEstimator.cpp calculate_js_divergence: log(P/M), log(Q/M) with
// P, Q, M > 0): the classic fdlibm reduction x = 2^k (1 + f), 1 + f in [sqrt(1/2), sqrt(2)), s = f / (2 + f),
// log(1 + f) = f - (f^2/2 - s (f^2/2 + R(s^2))) with fdlibm's degree-14 minimax R (Lg1..Lg7), and k ln2 split
// hi/lo.  ~30 fp64 ops against ~75 in the device library's log; <= 1 ulp from glibc (scripts/check_log_pos.cpp,
// tests/test_log_pos.py).  0 -> -inf, +inf -> +inf, NaN and negative inputs -> NaN, as log.
// ---------------------------------------------------------------------------------------------
LO_HD inline double log_pos(double x) {
    int k;
    double m = std::frexp(x, &k);                                // x = m 2^k, m in [1/2, 1) (denormals too)
    const bool lo_half = m < 0.70710678118654752440;
    m = lo_half ? m + m : m;
    k = lo_half ? k - 1 : k;
    const double f = m - 1.0;
    const double s = f / (2.0 + f);
    const double z = s * s, w = z * z;
    const double t1 = w * std::fma(w, std::fma(w, 1.531383769920937332e-01, 2.222219843214978396e-01),
                                   3.999999999940941908e-01);
    const double t2 = z * std::fma(w, std::fma(w, std::fma(w, 1.479819860511658591e-01, 1.818357216161805012e-01),
                                               2.857142874366239149e-01), 6.666666666666735130e-01);
    const double R = t2 + t1;
    const double hfsq = 0.5 * f * f;
    const double dk = static_cast<double>(k);
    const double r = dk * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + dk * 1.90821492927058770002e-10)) - f);
    const bool fin = x > 0.0 && x < INFINITY;
    return fin ? r : (x == 0.0 ? -INFINITY : (x > 0.0 ? x : NAN));
}

// ---------------------------------------------------------------------------------------------
// sinf / cosf as glibc 2.35 computes them on x86-64 with FMA (the reference's std::sin(float) / std::cos(float) in
// SO3::Exp, MathUtils.cpp:23-39): the optimized-routines algorithm (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c,
// sincosf.h) -- |y| < pi/4 by the top 12 bits: the degree-7 odd / degree-8 even polynomials in double; |y| < 120:
// reduce_fast by pi/2, the quadrant's sign and polynomial; the coefficients of __sincosf_table, the FMA build's
// contractions (glibc selects its -mfma variant by ifunc on such CPUs), rounded once to float.  Bit-identical to
// the host's sinf / cosf on every float in (1e-7, 120) (tests/test_sinf_restatement.py, exhaustive).  |y| >= 120,
// inf and NaN (glibc's large-argument reduction) fall back to the fp64 sin / cos rounded to float.
// ---------------------------------------------------------------------------------------------
struct SinCosTab {
    double c0, c1, s1, c2, s2, c3, s3, c4;
};
LO_HD inline uint32_t f32_top12(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return (u >> 20) & 0x7ffu;
}
LO_HD inline double sincosf_poly(double x, double x2, const SinCosTab& p, int n) {
    if ((n & 1) == 0) {
        const double x3 = x * x2, s1 = std::fma(x2, p.s3, p.s2), x7 = x3 * x2, s = std::fma(x3, p.s1, x);
        return std::fma(x7, s1, s);
    }
    const double x4 = x2 * x2, c2 = std::fma(x2, p.c4, p.c3), c1 = std::fma(x2, p.c1, p.c0), x6 = x4 * x2;
    const double c = std::fma(x4, p.c2, c1);
    return std::fma(x6, c2, c);
}
// which = 0: sinf, 1: cosf
LO_HD inline float sincosf_ref(float y, int which) {
    constexpr SinCosTab t0{1.0, -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, 0x1.55553e1068f19p-5,
                           0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16};
    constexpr SinCosTab t1{-1.0, 0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, -0x1.55553e1068f19p-5,
                           0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16};
    double x = y;
    const uint32_t a = f32_top12(y);
    if (a < f32_top12(0x1.921FB6p-1f)) {                          // |y| < pi/4
        const double x2 = x * x;
        if (a < f32_top12(0x1p-12f)) return which ? 1.0f : y;
        return static_cast<float>(sincosf_poly(x, x2, t0, which));
    }
    if (a < f32_top12(120.0f)) {                                  // reduce_fast
        const double r = x * 0x1.45F306DC9C883p+23;
        const int n = (static_cast<int32_t>(r) + 0x800000) >> 24;
        x = std::fma(-static_cast<double>(n), 0x1.921FB54442D18p0, x);
        const double sg = ((n & 3) == 0 || (n & 3) == 3) ? 1.0 : -1.0;
        return static_cast<float>(sincosf_poly(x * sg, x * x, (n & 2) ? t1 : t0, n ^ which));
    }
    return static_cast<float>(which ? std::cos(static_cast<double>(y)) : std::sin(static_cast<double>(y)));
}

// ---------------------------------------------------------------------------------------------
// Eigen JacobiSVD<Matrix3f>, square case (JacobiSVD.h compute(), real_2x2_jacobi_svd, makeJacobi)
// ---------------------------------------------------------------------------------------------
struct Rot { float c, s; };
LO_HD inline Rot rot_t(Rot r) { return {r.c, -r.s}; }
LO_HD inline Rot rot_mul(Rot a, Rot b) { return {a.c * b.c - a.s * b.s, a.c * b.s + a.s * b.c}; }
LO_HD inline void rotate(float& x, float& y, Rot r) {
    const float xi = x, yi = y;
    x = r.c * xi + r.s * yi;
    y = -r.s * xi + r.c * yi;
}
LO_HD inline Rot make_jacobi(float x, float y, float z) {
    const float deno = 2.0f * std::fabs(y);
    if (deno < FLT_MIN) return {1.0f, 0.0f};
    const float tau = (x - z) / deno;
    const float w = std::sqrt(tau * tau + 1.0f);
    const float t = tau > 0.0f ? 1.0f / (tau + w) : 1.0f / (tau - w);
    const float sgn = t > 0.0f ? 1.0f : -1.0f;
    const float n = 1.0f / std::sqrt(t * t + 1.0f);
    return {n, ((-sgn) * (y / std::fabs(y))) * std::fabs(t) * n};
}

// A row-major a[r][c]; U columns = left singular vectors, S descending.
LO_HD inline void jacobi_svd3(const float A[3][3], float U[3][3], float S[3], float Vout[3][3] = nullptr) {
    float scale = 0.0f;                                               // maxCoeff<PropagateNaN>
#pragma unroll
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) {
        const float v = std::fabs(A[r][c]);
        scale = (std::isnan(v) || std::isnan(scale)) ? NAN : std::max(scale, v);
    }
    float W[3][3], V[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) { U[r][c] = V[r][c] = (r == c) ? 1.0f : 0.0f; }
    if (!std::isfinite(scale)) {
        S[0] = S[1] = S[2] = NAN;
        if (Vout) for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) Vout[r][c] = V[r][c];
        return;
    }
    if (scale == 0.0f) scale = 1.0f;
#pragma unroll
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) W[r][c] = A[r][c] / scale;
    float maxDiag = std::max(std::fabs(W[0][0]), std::max(std::fabs(W[1][1]), std::fabs(W[2][2])));
    const float prec = 2.0f * FLT_EPSILON;
    bool done = false;
    for (int sweep = 0; !done && sweep < 1000; ++sweep) {
        done = true;
#pragma unroll
        for (int p = 1; p < 3; ++p) {
#pragma unroll
            for (int q = 0; q < p; ++q) {
                const float thr = std::max(FLT_MIN, prec * maxDiag);
                if (!(std::fabs(W[p][q]) > thr || std::fabs(W[q][p]) > thr)) continue;
                done = false;
                // real_2x2_jacobi_svd
                float m00 = W[p][p], m01 = W[p][q], m10 = W[q][p], m11 = W[q][q];
                Rot r1;
                const float t = m00 + m11, d = m10 - m01;
                if (std::fabs(d) < FLT_MIN) r1 = {1.0f, 0.0f};
                else {
                    const float u = t / d;
                    const float tmp = std::sqrt(1.0f + u * u);
                    r1 = {u / tmp, 1.0f / tmp};
                }
                rotate(m00, m10, r1);
                rotate(m01, m11, r1);
                const Rot jr = make_jacobi(m00, m01, m11);
                const Rot jl = rot_mul(r1, rot_t(jr));
#pragma unroll
                for (int i = 0; i < 3; ++i) rotate(W[p][i], W[q][i], jl);       // W.applyOnTheLeft(p,q,jl)
#pragma unroll
                for (int i = 0; i < 3; ++i) rotate(U[i][p], U[i][q], jl);       // U.applyOnTheRight(p,q,jl^T)
                const Rot jrt = rot_t(jr);
#pragma unroll
                for (int i = 0; i < 3; ++i) rotate(W[i][p], W[i][q], jrt);      // W.applyOnTheRight(p,q,jr)
#pragma unroll
                for (int i = 0; i < 3; ++i) rotate(V[i][p], V[i][q], jrt);
                maxDiag = std::max(maxDiag, std::max(std::fabs(W[p][p]), std::fabs(W[q][q])));
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float a = W[i][i];
        S[i] = std::fabs(a);
        if (a < 0.0f) for (int r = 0; r < 3; ++r) U[r][i] = -U[r][i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) S[i] *= scale;
#pragma unroll
    for (int i = 0; i < 3; ++i) {                                         // descending sort (first max)
        int pos = i;
#pragma unroll
        for (int k = i + 1; k < 3; ++k) if (S[k] > S[pos]) pos = k;
        if (S[pos] == 0.0f) break;
#pragma unroll
        for (int k = i + 1; k < 3; ++k) {                                  // swap with pos (compile-time indices:
            if (k != pos) continue;                                        // no scratch copy of U / V on the device)
            float tq = S[i]; S[i] = S[k]; S[k] = tq;
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                tq = U[r][i]; U[r][i] = U[r][k]; U[r][k] = tq;
                tq = V[r][i]; V[r][i] = V[r][k]; V[r][k] = tq;
            }
        }
    }
    if (Vout) for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) Vout[r][c] = V[r][c];
}

// Surfel fit of one L1 voxel (VoxelMap.cpp:211-243) over its m children's L0 centroids cs (xyz, child order): fp32
// mean and covariance in child order, JacobiSVD<Matrix3f>, normal = U.col(2); returns planarity = s2 / (s0 + 1e-6).
// One definition for the host map (lo_voxelmap.cpp) and the device fit (k_surfel_fit), so the two agree bit for bit.
LO_HD inline float surfel_fit(const float* cs, int m, float cen[3], float U[3][3]) {
    cen[0] = cen[1] = cen[2] = 0.0f;
    for (int q = 0; q < m; ++q) for (int a = 0; a < 3; ++a) cen[a] += cs[3 * q + a];
    const float mf = static_cast<float>(m);
    for (int a = 0; a < 3; ++a) cen[a] /= mf;
    float cov[3][3] = {{0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f}};
    for (int q = 0; q < m; ++q) {
        const float d[3] = {cs[3 * q] - cen[0], cs[3 * q + 1] - cen[1], cs[3 * q + 2] - cen[2]};
        for (int c = 0; c < 3; ++c) for (int r = 0; r < 3; ++r) cov[r][c] += d[c] * d[r];
    }
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) cov[r][c] /= mf;
    float S[3];
    jacobi_svd3(cov, U, S);
    return S[2] / (S[0] + 1e-6f);
}

// ---------------------------------------------------------------------------------------------
// SO3 / SE3f (MathUtils.h:57-168, MathUtils.cpp:41-99)
// ---------------------------------------------------------------------------------------------
LO_HD inline float dot3e(float a0, float a1, float a2, float b0, float b1, float b2) {   // Vector3f dot: e0 + (e1 + e2)
    const float e0 = a0 * b0, e1 = a1 * b1, e2 = a2 * b2;
    return e0 + (e1 + e2);
}
LO_HD inline void mul33e(const float A[3][3], const float B[3][3], float C[3][3]) {     // Matrix3f * Matrix3f
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) C[r][c] = dot3e(A[r][0], A[r][1], A[r][2], B[0][c], B[1][c], B[2][c]);
}
LO_HD inline float det3e(const float m[3][3]) {                                         // Eigen bruteforce_det3_helper order
    auto h = [&](int a, int b, int c) { return m[0][a] * (m[1][b] * m[2][c] - m[1][c] * m[2][b]); };
    return h(0, 1, 2) - h(1, 0, 2) + h(2, 0, 1);
}
// SO3(const Matrix3f&): U V^T of JacobiSVD, U.col(2) negated when det < 0 (MathUtils.cpp:86-99)
LO_HD inline void so3_project_svd(const float M[3][3], float R[3][3]) {
    float U[3][3], S[3], V[3][3], Vt[3][3];
    jacobi_svd3(M, U, S, V);
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) Vt[r][c] = V[c][r];
    mul33e(U, Vt, R);
    if (det3e(R) < 0.0f) {
        for (int r = 0; r < 3; ++r) U[r][2] *= -1.0f;
        mul33e(U, Vt, R);
    }
}
struct SE3f {
    float R[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    float t[3] = {0, 0, 0};
};
inline SE3f se3_from12(const float T[12]) {
    SE3f s;
    for (int r = 0; r < 3; ++r) { for (int c = 0; c < 3; ++c) s.R[r][c] = T[r * 4 + c]; s.t[r] = T[r * 4 + 3]; }
    return s;
}
inline void se3_to12(const SE3f& s, float T[12]) {
    for (int r = 0; r < 3; ++r) { for (int c = 0; c < 3; ++c) T[r * 4 + c] = s.R[r][c]; T[r * 4 + 3] = s.t[r]; }
}
// SE3::operator* (MathUtils.h:144-147): SO3(R1 R2), t1 + R1 t2
inline SE3f se3_mul(const SE3f& A, const SE3f& B) {
    SE3f o;
    float M[3][3];
    mul33e(A.R, B.R, M);
    so3_project_svd(M, o.R);
    for (int r = 0; r < 3; ++r) o.t[r] = A.t[r] + dot3e(A.R[r][0], A.R[r][1], A.R[r][2], B.t[0], B.t[1], B.t[2]);
    return o;
}
// SE3::Inverse (MathUtils.h:155-158): R_inv = SO3(R^T), t = R_inv * (-t)
inline SE3f se3_inv(const SE3f& A) {
    SE3f o;
    float Rt[3][3];
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) Rt[r][c] = A.R[c][r];
    so3_project_svd(Rt, o.R);
    for (int r = 0; r < 3; ++r) o.t[r] = dot3e(o.R[r][0], o.R[r][1], o.R[r][2], -A.t[0], -A.t[1], -A.t[2]);
    return o;
}
// |SO3::Log(R)| (MathUtils.cpp:41-84), kEps = 1e-6f
inline float so3_log_norm(const float m[3][3]) {
    const float trace = (m[0][0] + m[1][1]) + m[2][2];
    const float cos_theta = (trace - 1.0f) * 0.5f;
    const float theta = std::acos(std::max(-1.0f, std::min(1.0f, cos_theta)));
    float w[3];
    if (theta < 1e-6f) {
        w[0] = m[2][1] - 0.0f; w[1] = m[0][2] - 0.0f; w[2] = m[1][0] - 0.0f;          // Vee(R - I)
    } else {
        const float st = std::sin(theta);
        if (std::fabs(st) < 1e-6f) {
            int mi = 0;
            if (m[1][1] > m[0][0]) mi = 1;
            if (m[2][2] > m[mi][mi]) mi = 2;
            float axis[3];
            axis[mi] = std::sqrt((m[mi][mi] + 1.0f) * 0.5f);
            for (int i = 0; i < 3; ++i) if (i != mi) axis[i] = m[mi][i] / (2.0f * axis[mi]);
            const float sk[3] = {(m[2][1] - m[1][2]) * 0.5f, (m[0][2] - m[2][0]) * 0.5f, (m[1][0] - m[0][1]) * 0.5f};
            const float d = dot3e(axis[0], axis[1], axis[2], sk[0], sk[1], sk[2]);
            if (d < 0) for (float& a : axis) a = -a;
            for (int i = 0; i < 3; ++i) w[i] = axis[i] * theta;
        } else {
            const float f = theta / (2.0f * st);
            w[0] = f * (m[2][1] - m[1][2]); w[1] = f * (m[0][2] - m[2][0]); w[2] = f * (m[1][0] - m[0][1]);
        }
    }
    return std::sqrt(dot3e(w[0], w[1], w[2], w[0], w[1], w[2]));
}
// util::transform_point_cloud (PointCloudUtils.cpp:102-125): Matrix4f * Vector4f(x, y, z, 1), packet order
inline void transform_points(const SE3f& T, const float* in, size_t n, float* out) {
    for (size_t i = 0; i < n; ++i) {
        const float x = in[3 * i], y = in[3 * i + 1], z = in[3 * i + 2];
        for (int r = 0; r < 3; ++r) out[3 * i + r] = ((T.R[r][0] * x + T.R[r][1] * y) + T.R[r][2] * z) + T.t[r] * 1.0f;
    }
}

}  // namespace lo
