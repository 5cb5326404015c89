// lo_pgo.cpp — pose-graph optimisation (include/lo_pgo.h): the reference's PoseGraphOptimizer
// (src/optimization/PoseGraphOptimizer.cpp) restated on the host.
//
// The graph is small (one variable per keyframe: a few hundred to a few thousand) and solved once per loop closure,
// so this is host C++: the batch Gauss-Newton of PoseGraphOptimizer::optimize (:326-392) with the normal equations of
// buildLinearSystem (:394-469) assembled per 6x6 block and factored by an envelope (profile) LDL^T in keyframe
// order.  A keyframe chain keeps every row's envelope at one block; a loop closure i -> j widens row block j back to
// block i.  The reference factors with Eigen::SimplicialLDLT (AMD ordering); both are LDL^T without pivoting of the
// same SPD matrix, so they agree to rounding -- parity unpinned (Eigen absent here), see include/lo_pgo.h.
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstring>
#include <limits>
#include <map>
#include <mutex>
#include <set>
#include <vector>

#include "../../include/lo_icp.h"
#include "../../include/lo_pgo.h"
#include "lo_math.h"

namespace lo {
namespace pgo {

constexpr double kEpsLie = 1e-10;   // PoseGraphOptimizer.cpp:31

struct M3 {
    double a[3][3];
    static M3 zero() { M3 m; std::memset(m.a, 0, sizeof(m.a)); return m; }
    static M3 eye() { M3 m = zero(); m.a[0][0] = m.a[1][1] = m.a[2][2] = 1.0; return m; }
    double* operator[](int r) { return a[r]; }
    const double* operator[](int r) const { return a[r]; }
};
struct V3 { double v[3]; double& operator[](int i) { return v[i]; } double operator[](int i) const { return v[i]; } };

inline M3 mul(const M3& A, const M3& B) {
    M3 C;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) C[r][c] = A[r][0] * B[0][c] + A[r][1] * B[1][c] + A[r][2] * B[2][c];
    return C;
}
inline V3 mul(const M3& A, const V3& x) {
    V3 y;
    for (int r = 0; r < 3; ++r) y[r] = A[r][0] * x[0] + A[r][1] * x[1] + A[r][2] * x[2];
    return y;
}
inline M3 tr(const M3& A) { M3 T; for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) T[r][c] = A[c][r]; return T; }
inline M3 add(const M3& A, const M3& B) { M3 C; for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) C[r][c] = A[r][c] + B[r][c]; return C; }
inline M3 scale(double s, const M3& A) { M3 C; for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) C[r][c] = s * A[r][c]; return C; }
inline V3 sub(const V3& a, const V3& b) { return {{a[0] - b[0], a[1] - b[1], a[2] - b[2]}}; }
inline double norm(const V3& a) { return std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]); }
inline double det(const M3& m) {
    return m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) - m[1][0] * (m[0][1] * m[2][2] - m[0][2] * m[2][1]) +
           m[2][0] * (m[0][1] * m[1][2] - m[0][2] * m[1][1]);
}
// skew (PoseGraphOptimizer.cpp:36-42)
inline M3 skew(const V3& v) {
    M3 S = M3::zero();
    S[0][1] = -v[2]; S[0][2] = v[1];
    S[1][0] = v[2];  S[1][2] = -v[0];
    S[2][0] = -v[1]; S[2][1] = v[0];
    return S;
}

// Two-sided Jacobi SVD of a 3x3 (the scheme of Eigen::JacobiSVD, as lo_math.h's fp32 restatement), fp64.
inline void jacobi_svd3d(const M3& A, M3& U, double S[3], M3& V) {
    double sc = 0.0;
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) sc = std::max(sc, std::fabs(A[r][c]));
    U = M3::eye();
    V = M3::eye();
    if (!std::isfinite(sc)) { S[0] = S[1] = S[2] = NAN; return; }
    if (sc == 0.0) sc = 1.0;
    M3 W = scale(1.0 / sc, A);
    double maxDiag = std::max(std::fabs(W[0][0]), std::max(std::fabs(W[1][1]), std::fabs(W[2][2])));
    const double prec = 2.0 * DBL_EPSILON;
    auto rot = [](double& x, double& y, double c, double s) { const double xi = x, yi = y; x = c * xi + s * yi; y = -s * xi + c * yi; };
    bool done = false;
    for (int sweep = 0; !done && sweep < 1000; ++sweep) {
        done = true;
        for (int p = 1; p < 3; ++p)
            for (int q = 0; q < p; ++q) {
                const double thr = std::max(DBL_MIN, prec * maxDiag);
                if (!(std::fabs(W[p][q]) > thr || std::fabs(W[q][p]) > thr)) continue;
                done = false;
                double m00 = W[p][p], m01 = W[p][q], m10 = W[q][p], m11 = W[q][q];
                double c1 = 1.0, s1 = 0.0;
                const double t = m00 + m11, d = m10 - m01;
                if (std::fabs(d) >= DBL_MIN) { const double u = t / d, tmp = std::sqrt(1.0 + u * u); c1 = u / tmp; s1 = 1.0 / tmp; }
                rot(m00, m10, c1, s1);
                rot(m01, m11, c1, s1);
                double cj = 1.0, sj = 0.0;                                     // makeJacobi(m00, m01, m11)
                const double deno = 2.0 * std::fabs(m01);
                if (deno >= DBL_MIN) {
                    const double tau = (m00 - m11) / deno, w = std::sqrt(tau * tau + 1.0);
                    const double tt = tau > 0.0 ? 1.0 / (tau + w) : 1.0 / (tau - w);
                    const double sgn = tt > 0.0 ? 1.0 : -1.0, n = 1.0 / std::sqrt(tt * tt + 1.0);
                    cj = n;
                    sj = ((-sgn) * (m01 / std::fabs(m01))) * std::fabs(tt) * n;
                }
                const double cl = c1 * cj + s1 * sj, sl = c1 * (-sj) + s1 * cj;   // r1 * jr^T
                for (int i = 0; i < 3; ++i) rot(W[p][i], W[q][i], cl, sl);
                for (int i = 0; i < 3; ++i) rot(U[i][p], U[i][q], cl, sl);
                for (int i = 0; i < 3; ++i) rot(W[i][p], W[i][q], cj, -sj);
                for (int i = 0; i < 3; ++i) rot(V[i][p], V[i][q], cj, -sj);
                maxDiag = std::max(maxDiag, std::max(std::fabs(W[p][p]), std::fabs(W[q][q])));
            }
    }
    for (int i = 0; i < 3; ++i) {
        S[i] = std::fabs(W[i][i]);
        if (W[i][i] < 0.0) for (int r = 0; r < 3; ++r) U[r][i] = -U[r][i];
        S[i] *= sc;
    }
    for (int i = 0; i < 3; ++i) {
        int pos = i;
        for (int k = i + 1; k < 3; ++k) if (S[k] > S[pos]) pos = k;
        if (S[pos] == 0.0) break;
        if (pos != i) {
            std::swap(S[i], S[pos]);
            for (int r = 0; r < 3; ++r) { std::swap(U[r][i], U[r][pos]); std::swap(V[r][i], V[r][pos]); }
        }
    }
}

// SO3d(const Matrix3d&) (MathUtils.cpp:240-251): U V^T, U.col(2) negated when the determinant is negative
inline M3 so3d(const M3& M) {
    M3 U, V;
    double S[3];
    jacobi_svd3d(M, U, S, V);
    M3 R = mul(U, tr(V));
    if (det(R) < 0.0) {
        for (int r = 0; r < 3; ++r) U[r][2] = -U[r][2];
        R = mul(U, tr(V));
    }
    return R;
}

struct SE3d {
    M3 R = M3::eye();
    V3 t = {{0.0, 0.0, 0.0}};
};
// SE3d::FromMatrix (MathUtils.cpp:261-268): the rotation block projected onto SO(3)
inline SE3d from_matrix(const M3& R, const V3& t) { SE3d s; s.R = so3d(R); s.t = t; return s; }

// SO3_Logmap (:45-55)
inline V3 so3_log(const M3& R) {
    const double trc = R[0][0] + R[1][1] + R[2][2];
    const double theta = std::acos(std::clamp((trc - 1.0) / 2.0, -1.0, 1.0));
    const V3 v = {{R[2][1] - R[1][2], R[0][2] - R[2][0], R[1][0] - R[0][1]}};
    if (theta < kEpsLie) return {{v[0] / 2.0, v[1] / 2.0, v[2] / 2.0}};
    const double k = theta / (2.0 * std::sin(theta));
    return {{v[0] * k, v[1] * k, v[2] * k}};
}
// SO3_Expmap (:58-65)
inline M3 so3_exp(const V3& w) {
    const double theta = norm(w);
    if (theta < kEpsLie) return add(M3::eye(), skew(w));
    const M3 W = skew({{w[0] / theta, w[1] / theta, w[2] / theta}});
    return add(add(M3::eye(), scale(std::sin(theta), W)), scale(1.0 - std::cos(theta), mul(W, W)));
}
// SE3_Logmap (:81-97): [w (rot), u (trans)]
inline void se3_log(const M3& R, const V3& t, double xi[6]) {
    const V3 w = so3_log(R);
    const double theta = norm(w);
    for (int a = 0; a < 3; ++a) xi[a] = w[a];
    if (theta < kEpsLie) { for (int a = 0; a < 3; ++a) xi[3 + a] = t[a]; return; }
    const M3 W = skew({{w[0] / theta, w[1] / theta, w[2] / theta}});
    const double tan_half = std::tan(0.5 * theta);
    const V3 Wt = mul(W, t), WWt = mul(W, Wt);
    const double c = 1.0 - theta / (2.0 * tan_half);
    for (int a = 0; a < 3; ++a) xi[3 + a] = t[a] - (0.5 * theta) * Wt[a] + c * WWt[a];
}
// SE3_Expmap (:100-119)
inline void se3_exp(const double xi[6], M3& R, V3& t) {
    const V3 w = {{xi[0], xi[1], xi[2]}}, u = {{xi[3], xi[4], xi[5]}};
    R = so3_exp(w);
    const double theta = norm(w);
    if (theta < kEpsLie) { t = u; return; }
    const M3 W = skew(w);
    const double theta2 = theta * theta, s = std::sin(theta), c = std::cos(theta);
    const M3 V = add(add(M3::eye(), scale((1.0 - c) / theta2, W)), scale((theta - s) / (theta2 * theta), mul(W, W)));
    t = mul(V, u);
}

// Diagonal information (makeInformationMatrix, :607-621): [rot x3, trans x3]; sqrt_info = LLT(info).matrixL()^T,
// the element-wise square root for a diagonal matrix (PriorFactor / BetweenFactor constructors, .h:52-77).
struct SqrtInfo { double d[6]; };
inline SqrtInfo sqrt_info(double trans_noise, double rot_noise) {
    const double ti = 1.0 / (trans_noise * trans_noise), ri = 1.0 / (rot_noise * rot_noise);
    SqrtInfo s;
    for (int a = 0; a < 3; ++a) { s.d[a] = std::sqrt(ri); s.d[3 + a] = std::sqrt(ti); }
    return s;
}

struct Prior { int key; SE3d measured; SqrtInfo si; };
struct Between { int from, to; SE3d measured; SqrtInfo si; };

// Envelope LDL^T of the 6n x 6n normal matrix.  first[i] = first column of row i's envelope (the 6x6 block of the
// lowest-indexed variable row i's variable shares a factor with).
class Envelope {
  public:
    void reset(const std::vector<int>& first_var, int n_vars) {
        n_ = 6 * n_vars;
        first_.resize(n_);
        off_.resize(n_ + 1);
        size_t o = 0;
        for (int i = 0; i < n_; ++i) {
            first_[i] = 6 * first_var[i / 6];
            off_[i] = o;
            o += static_cast<size_t>(i - first_[i] + 1);
        }
        off_[n_] = o;
        a_.assign(o, 0.0);
    }
    double& at(int i, int j) { return a_[off_[i] + (j - first_[i])]; }      // j in [first[i], i]
    // lower-triangle accumulate of a 6x6 block (rows of variable vi, columns of vj, vj <= vi)
    void add_block(int vi, int vj, const double B[6][6]) {
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c < 6; ++c) {
                const int i = 6 * vi + r, j = 6 * vj + c;
                if (j <= i) at(i, j) += B[r][c];
            }
    }
    // in place: strictly-lower part -> L, diagonal -> D; false on a zero / non-finite pivot
    bool factor() {
        std::vector<double> t(n_);
        for (int i = 0; i < n_; ++i) {
            const int fi = first_[i];
            double* Ri = &a_[off_[i]];
            for (int j = fi; j < i; ++j) {
                const int lo = std::max(fi, first_[j]);
                const double* Rj = &a_[off_[j]];
                double s = Ri[j - fi];
                for (int k = lo; k < j; ++k) s -= t[k] * Rj[k - first_[j]];
                t[j] = s;                                            // L_ij * D_j
                Ri[j - fi] = s / Rj[j - first_[j]];
            }
            double d = Ri[i - fi];
            for (int k = fi; k < i; ++k) d -= t[k] * Ri[k - fi];
            if (!(d != 0.0) || !std::isfinite(d)) return false;
            Ri[i - fi] = d;
        }
        return true;
    }
    void solve(std::vector<double>& x) const {
        for (int i = 0; i < n_; ++i) {                               // L y = b
            const double* Ri = &a_[off_[i]];
            double s = x[i];
            for (int k = first_[i]; k < i; ++k) s -= Ri[k - first_[i]] * x[k];
            x[i] = s;
        }
        for (int i = 0; i < n_; ++i) x[i] /= a_[off_[i] + (i - first_[i])];
        for (int i = n_ - 1; i >= 0; --i) {                          // L^T x = z
            const double* Ri = &a_[off_[i]];
            const double xi = x[i];
            for (int k = first_[i]; k < i; ++k) x[k] -= Ri[k - first_[i]] * xi;
        }
    }

  private:
    int n_ = 0;
    std::vector<int> first_;
    std::vector<size_t> off_;
    std::vector<double> a_;
};

}  // namespace pgo
}  // namespace lo

using namespace lo::pgo;

struct lo_pgo {
    mutable std::mutex mu;
    std::vector<Prior> priors;
    std::vector<Between> betweens;
    std::map<int, SE3d> poses;
    std::vector<int> ids;
    std::set<int> id_set;
    std::map<int, int> index_of;
    size_t loop_count = 0, odom_count = 0;
    bool initialized = false;
    Envelope env;

    // toDouble (:597-600): Matrix4f cast to double, SE3d::FromMatrix
    static SE3d to_double(const float T[12]) {
        M3 R;
        V3 t;
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) R[r][c] = static_cast<double>(T[4 * r + c]);
            t[r] = static_cast<double>(T[4 * r + 3]);
        }
        return from_matrix(R, t);
    }
    // toFloat (:602-605): Matrix4d cast to float, SE3f::FromMatrix (SO3's fp32 SVD projection, lo_math.h)
    static void to_float(const SE3d& s, float T[12]) {
        float M[3][3], R[3][3];
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) M[r][c] = static_cast<float>(s.R[r][c]);
        lo::so3_project_svd(M, R);
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) T[4 * r + c] = R[r][c];
            T[4 * r + 3] = static_cast<float>(s.t[r]);
        }
    }

    // buildLinearSystem (:394-469): H = sum J^T J, b = -sum J^T e over whitened factors, H assembled in the
    // envelope, b dense
    void build(std::vector<double>& b) {
        const int n = static_cast<int>(ids.size());
        std::vector<int> fv(n);
        for (int v = 0; v < n; ++v) fv[v] = v;
        for (const Between& f : betweens) {
            const int lo = std::min(f.from, f.to), hi = std::max(f.from, f.to);
            fv[hi] = std::min(fv[hi], lo);
        }
        env.reset(fv, n);
        b.assign(6 * n, 0.0);
        for (const Prior& p : priors) {
            // computePriorError (:510-529): e = Log(measured^-1 T), J = I
            const SE3d& T = poses[ids[p.key]];
            const M3 Rmi = tr(p.measured.R);
            double e[6];
            se3_log(mul(Rmi, T.R), mul(Rmi, sub(T.t, p.measured.t)), e);
            double B[6][6] = {};
            for (int a = 0; a < 6; ++a) {
                B[a][a] = p.si.d[a] * p.si.d[a];
                b[6 * p.key + a] -= p.si.d[a] * (p.si.d[a] * e[a]);
            }
            env.add_block(p.key, p.key, B);
        }
        for (const Between& f : betweens) {
            // computeBetweenError (:471-508): hx = T_from^-1 T_to, e = Log(measured^-1 hx), J_to = I,
            // J_from = -Ad(hx^-1) with Ad = [R 0; [t]x R  R] ([rot, trans] order, SE3_AdjointMap :125-132)
            const SE3d& A = poses[ids[f.from]];
            const SE3d& Bp = poses[ids[f.to]];
            const M3 Rfi = tr(A.R);
            const M3 Rhx = mul(Rfi, Bp.R);
            const V3 thx = mul(Rfi, sub(Bp.t, A.t));
            const M3 Rmi = tr(f.measured.R);
            double e[6];
            se3_log(mul(Rmi, Rhx), mul(Rmi, sub(thx, f.measured.t)), e);
            const M3 Rinv = tr(Rhx);
            const V3 ti = mul(Rinv, thx);
            const V3 tinv = {{-ti[0], -ti[1], -ti[2]}};
            const M3 tR = mul(skew(tinv), Rinv);
            double Jf[6][6] = {};                                  // -Ad(hx^-1), whitened below
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) {
                    Jf[r][c] = -Rinv[r][c];
                    Jf[3 + r][c] = -tR[r][c];
                    Jf[3 + r][3 + c] = -Rinv[r][c];
                }
            double Jwf[6][6], ew[6];
            for (int r = 0; r < 6; ++r) {
                for (int c = 0; c < 6; ++c) Jwf[r][c] = f.si.d[r] * Jf[r][c];
                ew[r] = f.si.d[r] * e[r];
            }
            // H_ff = Jwf^T Jwf, H_tt = S^2, H_tf = S^T Jwf (= H_ft^T); b_f -= Jwf^T ew, b_t -= S ew
            double Hff[6][6], Htt[6][6] = {}, Htf[6][6];
            for (int r = 0; r < 6; ++r)
                for (int c = 0; c < 6; ++c) {
                    double s = 0.0;
                    for (int k = 0; k < 6; ++k) s += Jwf[k][r] * Jwf[k][c];
                    Hff[r][c] = s;
                    Htf[r][c] = f.si.d[r] * Jwf[r][c];
                }
            for (int a = 0; a < 6; ++a) Htt[a][a] = f.si.d[a] * f.si.d[a];
            env.add_block(f.from, f.from, Hff);
            env.add_block(f.to, f.to, Htt);
            if (f.to > f.from) env.add_block(f.to, f.from, Htf);
            else if (f.from > f.to) {
                double Hft[6][6];
                for (int r = 0; r < 6; ++r) for (int c = 0; c < 6; ++c) Hft[r][c] = Htf[c][r];
                env.add_block(f.from, f.to, Hft);
            } else {                                               // a self-loop: both cross blocks on the diagonal
                double Hs[6][6];
                for (int r = 0; r < 6; ++r) for (int c = 0; c < 6; ++c) Hs[r][c] = Htf[r][c] + Htf[c][r];
                env.add_block(f.to, f.to, Hs);
            }
            for (int r = 0; r < 6; ++r) {
                double s = 0.0;
                for (int k = 0; k < 6; ++k) s += Jwf[k][r] * ew[k];
                b[6 * f.from + r] -= s;
                b[6 * f.to + r] -= f.si.d[r] * ew[r];
            }
        }
    }

    // optimize (:326-392)
    bool optimize(int max_iterations, double threshold, int* iters_out) {
        const int n = static_cast<int>(ids.size());
        if (iters_out) *iters_out = 0;
        if (n == 0) return true;
        std::vector<double> dx;
        for (int it = 0; it < max_iterations; ++it) {
            build(dx);
            if (!env.factor()) return false;                       // "Cholesky decomposition failed"
            env.solve(dx);
            if (iters_out) *iters_out = it + 1;
            for (int v = 0; v < n; ++v) {
                SE3d& T = poses[ids[v]];
                M3 dR;
                V3 dt;
                se3_exp(&dx[6 * v], dR, dt);
                const M3 Rn = mul(T.R, dR);
                const V3 rt = mul(T.R, dt);
                const V3 tn = {{rt[0] + T.t[0], rt[1] + T.t[1], rt[2] + T.t[2]}};
                T = from_matrix(Rn, tn);
            }
            double s = 0.0;
            for (double v : dx) s += v * v;
            if (std::sqrt(s) < threshold) return true;
        }
        return false;
    }
};

extern "C" {

lo_pgo* lo_pgo_create(void) { return new lo_pgo(); }
void lo_pgo_destroy(lo_pgo* p) { delete p; }

int lo_pgo_add_first_keyframe(lo_pgo* p, int keyframe_id, const float pose[12]) {
    if (!p || !pose) return LO_ERR_ARG;
    std::lock_guard<std::mutex> g(p->mu);
    if (!p->ids.empty()) return 0;
    const SE3d d = lo_pgo::to_double(pose);
    p->priors.push_back({0, d, sqrt_info(1e-4, 1e-4)});
    p->poses[keyframe_id] = d;
    p->ids.push_back(keyframe_id);
    p->id_set.insert(keyframe_id);
    p->index_of[keyframe_id] = 0;
    p->initialized = true;
    return 1;
}

int lo_pgo_add_keyframe_with_odom(lo_pgo* p, int prev_keyframe_id, int curr_keyframe_id, const float curr_pose[12],
                                  const float relative_pose[12], double odom_trans_noise, double odom_rot_noise) {
    if (!p || !curr_pose || !relative_pose) return LO_ERR_ARG;
    std::lock_guard<std::mutex> g(p->mu);
    if (p->id_set.count(curr_keyframe_id)) return 1;
    const SE3d cur = lo_pgo::to_double(curr_pose), rel = lo_pgo::to_double(relative_pose);
    const int idx = static_cast<int>(p->ids.size());
    if (p->id_set.count(prev_keyframe_id)) {
        p->betweens.push_back({p->index_of[prev_keyframe_id], idx, rel, sqrt_info(odom_trans_noise, odom_rot_noise)});
    } else {
        p->priors.push_back({idx, cur, sqrt_info(0.5, 0.1)});   // loose prior (:226-230)
    }
    p->poses[curr_keyframe_id] = cur;
    p->ids.push_back(curr_keyframe_id);
    p->id_set.insert(curr_keyframe_id);
    p->index_of[curr_keyframe_id] = idx;
    p->odom_count++;
    return 1;
}

int lo_pgo_add_loop_and_optimize(lo_pgo* p, int from_keyframe_id, int to_keyframe_id, const float relative_pose[12],
                                 double loop_trans_noise, double loop_rot_noise, int* converged, int* iterations,
                                 double* ms) {
    if (!p || !relative_pose) return LO_ERR_ARG;
    std::lock_guard<std::mutex> g(p->mu);
    if (!p->id_set.count(from_keyframe_id) || !p->id_set.count(to_keyframe_id)) return 0;
    p->betweens.push_back({p->index_of[from_keyframe_id], p->index_of[to_keyframe_id],
                           lo_pgo::to_double(relative_pose), sqrt_info(loop_trans_noise, loop_rot_noise)});
    const auto t0 = std::chrono::steady_clock::now();
    int it = 0;
    const bool conv = p->optimize(10, 1e-6, &it);
    const double dt = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    p->loop_count++;
    if (converged) *converged = conv ? 1 : 0;
    if (iterations) *iterations = it;
    if (ms) *ms = dt;
    return 1;
}

int lo_pgo_get_optimized_pose(const lo_pgo* p, int keyframe_id, float pose[12]) {
    if (!p || !pose) return LO_ERR_ARG;
    std::lock_guard<std::mutex> g(p->mu);
    const auto it = p->poses.find(keyframe_id);
    if (it == p->poses.end()) return 0;
    lo_pgo::to_float(it->second, pose);
    return 1;
}

size_t lo_pgo_get_all_optimized_poses(const lo_pgo* p, int* ids, float* poses, size_t cap) {
    if (!p) return 0;
    std::lock_guard<std::mutex> g(p->mu);
    size_t c = 0;
    for (const auto& kv : p->poses) {
        if (c >= cap) break;
        if (ids) ids[c] = kv.first;
        if (poses) lo_pgo::to_float(kv.second, poses + 12 * c);
        ++c;
    }
    return c;
}

int lo_pgo_has_keyframe(const lo_pgo* p, int keyframe_id) {
    if (!p) return LO_ERR_ARG;
    std::lock_guard<std::mutex> g(p->mu);
    return p->id_set.count(keyframe_id) ? 1 : 0;
}
size_t lo_pgo_keyframe_count(const lo_pgo* p) {
    if (!p) return 0;
    std::lock_guard<std::mutex> g(p->mu);
    return p->ids.size();
}
size_t lo_pgo_loop_closure_count(const lo_pgo* p) {
    if (!p) return 0;
    std::lock_guard<std::mutex> g(p->mu);
    return p->loop_count;
}
void lo_pgo_clear(lo_pgo* p) {
    if (!p) return;
    std::lock_guard<std::mutex> g(p->mu);
    p->priors.clear();
    p->betweens.clear();
    p->poses.clear();
    p->ids.clear();
    p->id_set.clear();
    p->index_of.clear();
    p->loop_count = p->odom_count = 0;
    p->initialized = false;
}

}  // extern "C"
