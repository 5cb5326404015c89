/*
 * lo_oracle.cpp — CPU ORACLE for the ICP hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * A single-threaded restatement of the reference (SiarheiHerasiuta/lidar_odometry) point-to-plane
 * ICP step, written from the reference source without Eigen.  It is the checker for the HIP product
 * (tests/), the `cpu_baseline` leg of bench.py and nothing else: the product never links or calls it.
 *
 * Faithfulness rules followed here:
 *  - every floating-point expression keeps the reference's precision (fp32 vs fp64) and the
 *    operation order that Eigen 3.4 produces for fixed-size objects on x86-64/SSE2 without FMA:
 *      Matrix4f*Vector4f  (packet path)       : ((c0*x + c1*y) + c2*z) + c3*w
 *      Matrix3f*Vector3f, Vector3f.dot/norm   : e0 + (e1 + e2)        (redux_novec_unroller)
 *      Vector3d.dot                           : (e0 + e1) + e2         (Packet2d + tail)
 *    The library is compiled with -O3 -ffp-contract=off and no -march (the reference's Release
 *    flags have no -march, CMakeLists.txt:19-21, so no FMA is ever emitted there).
 *  - unordered_dense containers are restated as "dense value vector in insertion order, erase moves the
 *    last value into the hole" (unordered_dense.h do_erase) — the only property the reference's results
 *    depend on (iteration order).
 *  - PKO uses the real libstdc++ std::mt19937 / std::shuffle / std::uniform_int_distribution, exactly as
 *    AdaptiveMEstimator.cpp does.
 *
 * Parity status: PKO pinned against reference golden vectors (tests/golden/pko_golden.json, produced by
 * oracle/ref/pko_golden.cpp linked with the reference's own AdaptiveMEstimator.cpp).  Eigen-dependent
 * pieces (JacobiSVD, LDLT, SE3, surfel PCA, correspondences) are parity UNPINNED against reference
 * binaries (Eigen absent, reference unbuildable here).
 */
#include "lo_oracle.h"

#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <numeric>
#include <random>
#include <utility>
#include <vector>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

namespace orc {

/* ===================================================================================== */
/*  Small fixed-size algebra with Eigen's evaluation order                                */
/* ===================================================================================== */

struct M3 { float a[3][3]; };   // a[row][col]

static inline float dot3f(float a0, float a1, float a2, float b0, float b1, float b2) {
    float e0 = a0 * b0, e1 = a1 * b1, e2 = a2 * b2;
    return e0 + (e1 + e2);
}
static inline double dot3d(double a0, double a1, double a2, double b0, double b1, double b2) {
    double e0 = a0 * b0, e1 = a1 * b1, e2 = a2 * b2;
    return (e0 + e1) + e2;
}
static inline float norm3f(const float v[3]) { return std::sqrt(dot3f(v[0], v[1], v[2], v[0], v[1], v[2])); }

static M3 eye3() { M3 m; for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) m.a[r][c] = (r == c) ? 1.0f : 0.0f; return m; }

// Matrix3f * Matrix3f (lazy coeff-based product, MathUtils.h:81-83)
static M3 mul33(const M3& A, const M3& B) {
    M3 C;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            C.a[r][c] = dot3f(A.a[r][0], A.a[r][1], A.a[r][2], B.a[0][c], B.a[1][c], B.a[2][c]);
    return C;
}
// Matrix3f * Vector3f
static inline void mul3v(const M3& A, const float v[3], float out[3]) {
    for (int r = 0; r < 3; ++r) out[r] = dot3f(A.a[r][0], A.a[r][1], A.a[r][2], v[0], v[1], v[2]);
}

/* ---- JacobiSVD<Matrix3f> (Eigen 3.4 JacobiSVD::compute, square case, no preconditioner) ---- */
struct JRot { float c, s; };

// makeJacobi(x, y, z) (Eigen/src/Jacobi/Jacobi.h)
static JRot make_jacobi(float x, float y, float z) {
    JRot j;
    float deno = 2.0f * std::fabs(y);
    if (deno < FLT_MIN) { j.c = 1.0f; j.s = 0.0f; return j; }
    float tau = (x - z) / deno;
    float w = std::sqrt(tau * tau + 1.0f);
    float t = (tau > 0.0f) ? 1.0f / (tau + w) : 1.0f / (tau - w);
    float sign_t = t > 0.0f ? 1.0f : -1.0f;
    float n = 1.0f / std::sqrt(t * t + 1.0f);
    j.s = ((-sign_t) * (y / std::fabs(y))) * std::fabs(t) * n;
    j.c = n;
    return j;
}
// rot1 * rot2 (JacobiRotation::operator*)
static JRot jmul(JRot a, JRot b) { JRot r; r.c = a.c * b.c - a.s * b.s; r.s = a.c * b.s + a.s * b.c; return r; }
static JRot jtrans(JRot a) { JRot r; r.c = a.c; r.s = -a.s; return r; }
// apply_rotation_in_the_plane(x, y, j): x' = c x + s y ; y' = -s x + c y
static inline void rot_pair(float& x, float& y, JRot j) {
    float xi = x, yi = y;
    x = j.c * xi + j.s * yi;
    y = -j.s * xi + j.c * yi;
}
static void apply_left(M3& M, int p, int q, JRot j) { for (int i = 0; i < 3; ++i) rot_pair(M.a[p][i], M.a[q][i], j); }
static void apply_right(M3& M, int p, int q, JRot j) { JRot t = jtrans(j); for (int i = 0; i < 3; ++i) rot_pair(M.a[i][p], M.a[i][q], t); }

static void real_2x2_jacobi_svd(const M3& W, int p, int q, JRot* jl, JRot* jr) {
    float m00 = W.a[p][p], m01 = W.a[p][q], m10 = W.a[q][p], m11 = W.a[q][q];
    JRot rot1;
    float t = m00 + m11;
    float d = m10 - m01;
    if (std::fabs(d) < FLT_MIN) { rot1.s = 0.0f; rot1.c = 1.0f; }
    else {
        float u = t / d;
        float tmp = std::sqrt(1.0f + u * u);
        rot1.s = 1.0f / tmp;
        rot1.c = u / tmp;
    }
    // m.applyOnTheLeft(0,1,rot1)
    rot_pair(m00, m10, rot1);
    rot_pair(m01, m11, rot1);
    *jr = make_jacobi(m00, m01, m11);
    *jl = jmul(rot1, jtrans(*jr));
}

// Returns 0 on success, -1 on non-finite input.  U, V full; S descending.
static int jacobi_svd3(const M3& A, M3& U, float S[3], M3& V) {
    float scale = 0.0f;
    bool nan = false;
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) {
        float v = std::fabs(A.a[r][c]);
        if (std::isnan(v)) nan = true;
        if (v > scale) scale = v;
    }
    if (nan || !std::isfinite(scale)) { U = eye3(); V = eye3(); S[0] = S[1] = S[2] = NAN; return -1; }
    if (scale == 0.0f) scale = 1.0f;
    M3 W;
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) W.a[r][c] = A.a[r][c] / scale;
    U = eye3(); V = eye3();
    const float precision = 2.0f * FLT_EPSILON;
    const float considerAsZero = FLT_MIN;
    float maxDiag = std::max(std::fabs(W.a[0][0]), std::max(std::fabs(W.a[1][1]), std::fabs(W.a[2][2])));
    // Eigen maxCoeff over |diag|: strict '>' visitor; with no NaN same as max.
    bool finished = false;
    int sweeps = 0;
    while (!finished && sweeps < 1000) {
        finished = true;
        ++sweeps;
        for (int p = 1; p < 3; ++p) {
            for (int q = 0; q < p; ++q) {
                float threshold = std::max(considerAsZero, precision * maxDiag);
                if (std::fabs(W.a[p][q]) > threshold || std::fabs(W.a[q][p]) > threshold) {
                    finished = false;
                    JRot jl, jr;
                    real_2x2_jacobi_svd(W, p, q, &jl, &jr);
                    apply_left(W, p, q, jl);
                    apply_right(U, p, q, jtrans(jl));
                    apply_right(W, p, q, jr);
                    apply_right(V, p, q, jr);
                    maxDiag = std::max(maxDiag, std::max(std::fabs(W.a[p][p]), std::fabs(W.a[q][q])));
                }
            }
        }
    }
    for (int i = 0; i < 3; ++i) {
        float a = W.a[i][i];
        S[i] = std::fabs(a);
        if (a < 0.0f) for (int r = 0; r < 3; ++r) U.a[r][i] = -U.a[r][i];
    }
    for (int i = 0; i < 3; ++i) S[i] *= scale;
    for (int i = 0; i < 3; ++i) {
        int pos = i;
        float mx = S[i];
        for (int k = i + 1; k < 3; ++k) if (S[k] > mx) { mx = S[k]; pos = k; }
        if (mx == 0.0f) break;
        if (pos != i) {
            std::swap(S[i], S[pos]);
            for (int r = 0; r < 3; ++r) { std::swap(U.a[r][i], U.a[r][pos]); std::swap(V.a[r][i], V.a[r][pos]); }
        }
    }
    return 0;
}

// Eigen 3x3 determinant (bruteforce_det3_helper order)
static float det3(const M3& m) {
    auto h = [&](int a, int b, int c) { return m.a[0][a] * (m.a[1][b] * m.a[2][c] - m.a[1][c] * m.a[2][b]); };
    return h(0, 1, 2) - h(1, 0, 2) + h(2, 0, 1);
}

// SO3(const Matrix3f&) — MathUtils.cpp:86-99
static M3 so3_normalize(const M3& R) {
    M3 U, V; float S[3];
    jacobi_svd3(R, U, S, V);
    M3 Vt; for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) Vt.a[r][c] = V.a[c][r];
    M3 out = mul33(U, Vt);
    if (det3(out) < 0.0f) {
        for (int r = 0; r < 3; ++r) U.a[r][2] *= -1.0f;
        out = mul33(U, Vt);
    }
    return out;
}

static M3 hat3(const float v[3]) {
    M3 S;
    S.a[0][0] = 0.0f;  S.a[0][1] = -v[2]; S.a[0][2] = v[1];
    S.a[1][0] = v[2];  S.a[1][1] = 0.0f;  S.a[1][2] = -v[0];
    S.a[2][0] = -v[1]; S.a[2][1] = v[0];  S.a[2][2] = 0.0f;
    return S;
}

// SO3::Exp — MathUtils.cpp:23-39 (kEps = 1e-6f, MathUtils.h:40)
static M3 so3_exp(const float w[3]) {
    const float theta = norm3f(w);
    if (theta < 1e-6f) {
        M3 H = hat3(w), R = eye3();
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) R.a[r][c] = R.a[r][c] + H.a[r][c];
        return so3_normalize(R);
    }
    const float theta_inv = 1.0f / theta;
    float k[3] = {w[0] * theta_inv, w[1] * theta_inv, w[2] * theta_inv};
    M3 K = hat3(k);
    float s = std::sin(theta), omc = 1.0f - std::cos(theta);
    M3 sK;  for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) sK.a[r][c] = omc * K.a[r][c];
    M3 KK = mul33(sK, K);   // ((1-cos)*K)*K, lazy product of the scaled expression
    M3 R;
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c)
        R.a[r][c] = ((r == c ? 1.0f : 0.0f) + s * K.a[r][c]) + KK.a[r][c];
    return so3_normalize(R);
}

struct SE3 { M3 R; float t[3]; };
static SE3 se3_from12(const float T[12]) {
    SE3 s;
    for (int r = 0; r < 3; ++r) { for (int c = 0; c < 3; ++c) s.R.a[r][c] = T[r * 4 + c]; s.t[r] = T[r * 4 + 3]; }
    return s;
}
static void se3_to12(const SE3& s, float T[12]) {
    for (int r = 0; r < 3; ++r) { for (int c = 0; c < 3; ++c) T[r * 4 + c] = s.R.a[r][c]; T[r * 4 + 3] = s.t[r]; }
}
// SE3::operator* — MathUtils.h:144-147
static SE3 se3_mul(const SE3& A, const SE3& B) {
    SE3 o;
    o.R = so3_normalize(mul33(A.R, B.R));
    float Rt[3]; mul3v(A.R, B.t, Rt);
    for (int i = 0; i < 3; ++i) o.t[i] = A.t[i] + Rt[i];
    return o;
}

/* ---- LDLT (Eigen ldlt_inplace<Lower>::unblocked + LDLT::_solve_impl), fp32 6x6 ---- */
static void ldlt6_solve(const float Hin[36], const float b[6], float x[6]) {
    float m[6][6];
    for (int r = 0; r < 6; ++r) for (int c = 0; c < 6; ++c) m[r][c] = Hin[r * 6 + c];
    int transp[6];
    float temp[6];
    const int size = 6;
    bool zero_all = false;
    for (int k = 0; k < size; ++k) {
        int big = k; float bv = std::fabs(m[k][k]);
        for (int i = k + 1; i < size; ++i) if (std::fabs(m[i][i]) > bv) { bv = std::fabs(m[i][i]); big = i; }
        transp[k] = big;
        if (k != big) {
            for (int j = 0; j < k; ++j) std::swap(m[k][j], m[big][j]);
            for (int i = big + 1; i < size; ++i) std::swap(m[i][k], m[i][big]);
            std::swap(m[k][k], m[big][big]);
            for (int i = k + 1; i < big; ++i) { float tmp = m[i][k]; m[i][k] = m[big][i]; m[big][i] = tmp; }
        }
        int rs = size - k - 1;
        if (k > 0) {
            for (int j = 0; j < k; ++j) temp[j] = m[j][j] * m[k][j];
            float acc = 0.0f; for (int j = 0; j < k; ++j) acc += m[k][j] * temp[j];
            m[k][k] -= acc;
            for (int i = k + 1; i < size; ++i) { float a = 0.0f; for (int j = 0; j < k; ++j) a += m[i][j] * temp[j]; m[i][k] -= a; }
        }
        float akk = m[k][k];
        bool valid = std::fabs(akk) > 0.0f;
        if (k == 0 && !valid) { zero_all = true; break; }
        if (rs > 0 && valid) for (int i = k + 1; i < size; ++i) m[i][k] /= akk;
    }
    if (zero_all) { for (int i = 0; i < 6; ++i) x[i] = 0.0f; return; }
    float d[6];
    for (int i = 0; i < 6; ++i) d[i] = b[i];
    for (int k = 0; k < size; ++k) if (transp[k] != k) std::swap(d[k], d[transp[k]]);
    for (int i = 0; i < size; ++i) { float a = 0.0f; for (int j = 0; j < i; ++j) a += m[i][j] * d[j]; d[i] -= a; }
    for (int i = 0; i < size; ++i) { if (std::fabs(m[i][i]) > FLT_MIN) d[i] /= m[i][i]; else d[i] = 0.0f; }
    for (int i = size - 1; i >= 0; --i) { float a = 0.0f; for (int j = i + 1; j < size; ++j) a += m[j][i] * d[j]; d[i] -= a; }
    for (int k = size - 1; k >= 0; --k) if (transp[k] != k) std::swap(d[k], d[transp[k]]);
    for (int i = 0; i < 6; ++i) x[i] = d[i];
}

/* ===================================================================================== */
/*  Dense hash containers (unordered_dense semantics: insertion-ordered values,          */
/*  erase = move last value into the hole)                                                */
/* ===================================================================================== */

struct VKey { int x, y, z; bool operator==(const VKey& o) const { return x == o.x && y == o.y && z == o.z; } };

static inline uint64_t expand_bits21(int32_t v) {
    uint64_t x = static_cast<uint64_t>(v + (1 << 20)) & 0x1fffffULL;
    x = (x | (x << 32)) & 0x1f00000000ffffULL;
    x = (x | (x << 16)) & 0x1f0000ff0000ffULL;
    x = (x | (x << 8)) & 0x100f00f00f00f00fULL;
    x = (x | (x << 4)) & 0x10c30c30c30c30c3ULL;
    x = (x | (x << 2)) & 0x1249249249249249ULL;
    return x;
}
// VoxelKeyHash (VoxelMap.h:166-183) followed by unordered_dense's wyhash mix for non-avalanching hashes
static inline uint64_t vkey_hash(const VKey& k) {
    uint64_t morton = expand_bits21(k.x) | (expand_bits21(k.y) << 1) | (expand_bits21(k.z) << 2);
    __uint128_t r = static_cast<__uint128_t>(morton) * 0x9E3779B97F4A7C15ULL;
    return static_cast<uint64_t>(r) ^ static_cast<uint64_t>(r >> 64);
}

template <typename V>
struct DenseMap {
    std::vector<std::pair<VKey, V>> vals;
    std::vector<uint32_t> buckets;   // 0 = empty, else value index + 1
    uint64_t mask = 0;

    DenseMap() { rehash(16); }
    void rehash(size_t cap) {
        buckets.assign(cap, 0u);
        mask = cap - 1;
        for (size_t i = 0; i < vals.size(); ++i) place(static_cast<uint32_t>(i));
    }
    void place(uint32_t vi) {
        uint64_t b = vkey_hash(vals[vi].first) & mask;
        while (buckets[b]) b = (b + 1) & mask;
        buckets[b] = vi + 1;
    }
    int64_t find_bucket(const VKey& k) const {
        uint64_t b = vkey_hash(k) & mask;
        while (buckets[b]) {
            if (vals[buckets[b] - 1].first == k) return static_cast<int64_t>(b);
            b = (b + 1) & mask;
        }
        return -1;
    }
    V* find(const VKey& k) { int64_t b = find_bucket(k); return b < 0 ? nullptr : &vals[buckets[b] - 1].second; }
    const V* find(const VKey& k) const { int64_t b = find_bucket(k); return b < 0 ? nullptr : &vals[buckets[b] - 1].second; }
    V& operator[](const VKey& k) {
        int64_t b = find_bucket(k);
        if (b >= 0) return vals[buckets[b] - 1].second;
        if ((vals.size() + 1) * 5 > buckets.size() * 4) rehash(buckets.size() * 2);   // max load 0.8
        vals.emplace_back(k, V());
        place(static_cast<uint32_t>(vals.size() - 1));
        return vals.back().second;
    }
    bool insert_key(const VKey& k) {   // set semantics
        if (find_bucket(k) >= 0) return false;
        (*this)[k];
        return true;
    }
    bool erase(const VKey& k) {
        int64_t bi = find_bucket(k);
        if (bi < 0) return false;
        uint64_t b = static_cast<uint64_t>(bi);
        uint32_t vi = buckets[b] - 1;
        // backward-shift deletion (linear probing)
        buckets[b] = 0;
        uint64_t j = (b + 1) & mask;
        while (buckets[j]) {
            uint64_t home = vkey_hash(vals[buckets[j] - 1].first) & mask;
            bool move = ((j - home) & mask) >= ((j - b) & mask) ? true : false;
            // move if the hole lies cyclically in [home, j)
            if (((j - home) & mask) >= ((j - b) & mask)) { buckets[b] = buckets[j]; buckets[j] = 0; b = j; }
            (void)move;
            j = (j + 1) & mask;
        }
        uint32_t last = static_cast<uint32_t>(vals.size() - 1);
        if (vi != last) {
            int64_t lb = find_bucket(vals[last].first);
            vals[vi] = std::move(vals[last]);
            buckets[lb] = vi + 1;
        }
        vals.pop_back();
        return true;
    }
    size_t size() const { return vals.size(); }
    bool empty() const { return vals.empty(); }
    void clear() { vals.clear(); rehash(16); }
};

struct Empty {};
using KeySet = DenseMap<Empty>;

/* ===================================================================================== */
/*  VoxelMap (VoxelMap.cpp)                                                               */
/* ===================================================================================== */

struct L0Node { float c[3] = {0.0f, 0.0f, 0.0f}; int hit_count = 1; int point_count = 0; };
struct L1Node {
    KeySet children;
    bool has_surfel = false;
    float normal[3] = {0.0f, 0.0f, 0.0f};
    float centroid[3] = {0.0f, 0.0f, 0.0f};
    float planarity = 1.0f;
    int last_child_count = 0;
};


/* ---- nanoflann 1.7.1 KDTreeSingleIndexAdaptor, restated (util::KdTree, PointCloudUtils.h:370-423, built by
 * VoxelMap::RebuildKdTree :420-438; thirdparty/nanoflann/nanoflann.hpp) ----
 * Leaf size 10, DIM 3, L2_Simple_Adaptor<float>: every quantity is fp32 as nanoflann computes it.
 *  build   computeBoundingBox (:1845-1880) over vAcc_ = iota; divideTree (:1149-1210): a range of <= 10 points is
 *          a leaf whose box is its points' min / max; otherwise middleSplit_ (:1320-1370) picks, among the axes whose
 *          inherited box span is >= (1 - 1e-5) * the largest span, the one with the largest point spread, cuts at
 *          the box midpoint clamped to the points' [min, max], and planeSplit (:1382-1427) partitions vAcc_ in place
 *          (two Hoare-style passes); the split index is lim1 / lim2 / count / 2 as nanoflann balances it; divlow /
 *          divhigh are the children's actual extents in the cut axis, the node box the union of its children's.
 *  search  findNeighbors (:1708-1730): per-axis squared distances to the root box, then searchLevel (:1885-1960):
 *          a leaf adds each point with dist < the worstDist read at leaf entry; an inner node descends first into
 *          child1 if (q - divlow) + (q - divhigh) < 0, else child2, and visits the other child when the
 *          incrementally updated fp32 box distance is <= worstDist.  KNNResultSet (:199-282) insertion-sorts and
 *          keeps the earlier-visited point among equal distances (NANOFLANN_FIRST_MATCH is not defined).
 * So the result is the 5 smallest by (fp32 distance, visit order) -- visit_before() states that order directly:
 * leaves in the near-child-first DFS order of the query, points of one leaf in vAcc_ order.  knn_brute() (an
 * exhaustive scan ranked by that order) equals the tree search except where the tree's fp32 box-distance bound
 * rounds above a point's own fp32 distance (never seen on the fixtures; tests/test_oracle.py checks both against
 * nanoflann itself, tests/golden/knn_*.npz). */
struct KdTree3 {
    struct Node {
        int child1 = -1, child2 = -1;         // -1: leaf
        size_t left = 0, right = 0;           // vAcc_ range; inner nodes: [left, mid) -> child1, [mid, right) -> child2
        size_t mid = 0;
        int divfeat = 0;
        float divlow = 0.0f, divhigh = 0.0f;
    };
    struct Box { float low[3], high[3]; };
    std::vector<float> pts;                  // xyz by original index (GetPointCloud order)
    std::vector<uint32_t> vacc;              // vAcc_
    std::vector<uint32_t> vpos;              // original index -> position in vAcc_
    std::vector<Node> nodes;
    Box root_bbox{};
    int root = -1;

    float get(uint32_t i, int d) const { return pts[3 * static_cast<size_t>(i) + d]; }

    void build(const std::vector<float>& cloud) {
        pts = cloud;
        const size_t m = cloud.size() / 3;
        vacc.resize(m);
        for (size_t i = 0; i < m; ++i) vacc[i] = static_cast<uint32_t>(i);
        nodes.clear();
        root = -1;
        if (m == 0) { vpos.clear(); return; }
        for (int d = 0; d < 3; ++d) root_bbox.low[d] = root_bbox.high[d] = get(vacc[0], d);
        for (size_t k = 1; k < m; ++k)
            for (int d = 0; d < 3; ++d) {
                const float v = get(vacc[k], d);
                if (v < root_bbox.low[d]) root_bbox.low[d] = v;
                if (v > root_bbox.high[d]) root_bbox.high[d] = v;
            }
        Box bb = root_bbox;
        root = divide(0, m, bb);
        vpos.assign(m, 0);
        for (size_t i = 0; i < m; ++i) vpos[vacc[i]] = static_cast<uint32_t>(i);
    }

    int divide(size_t left, size_t right, Box& bbox) {
        const int id = static_cast<int>(nodes.size());
        nodes.emplace_back();
        if (right - left <= 10) {
            nodes[id].left = left;
            nodes[id].right = right;
            for (int d = 0; d < 3; ++d) bbox.low[d] = bbox.high[d] = get(vacc[left], d);
            for (size_t k = left + 1; k < right; ++k)
                for (int d = 0; d < 3; ++d) {
                    const float v = get(vacc[k], d);
                    if (bbox.low[d] > v) bbox.low[d] = v;
                    if (bbox.high[d] < v) bbox.high[d] = v;
                }
            return id;
        }
        size_t idx;
        int cutfeat;
        float cutval;
        middle_split(left, right - left, idx, cutfeat, cutval, bbox);
        Box lb = bbox;
        lb.high[cutfeat] = cutval;
        const int c1 = divide(left, left + idx, lb);
        Box rb = bbox;
        rb.low[cutfeat] = cutval;
        const int c2 = divide(left + idx, right, rb);
        Node& nd = nodes[id];
        nd.child1 = c1;
        nd.child2 = c2;
        nd.left = left;
        nd.right = right;
        nd.mid = left + idx;
        nd.divfeat = cutfeat;
        nd.divlow = lb.high[cutfeat];
        nd.divhigh = rb.low[cutfeat];
        for (int d = 0; d < 3; ++d) {
            bbox.low[d] = std::min(lb.low[d], rb.low[d]);
            bbox.high[d] = std::max(lb.high[d], rb.high[d]);
        }
        return id;
    }

    void middle_split(size_t ind, size_t count, size_t& index, int& cutfeat, float& cutval, const Box& bbox) {
        const float EPS = static_cast<float>(0.00001);
        float max_span = bbox.high[0] - bbox.low[0];
        for (int i = 1; i < 3; ++i) {
            const float span = bbox.high[i] - bbox.low[i];
            if (span > max_span) max_span = span;
        }
        float max_spread = -1.0f;
        cutfeat = 0;
        float min_elem = 0.0f, max_elem = 0.0f;
        for (int i = 0; i < 3; ++i) {
            const float span = bbox.high[i] - bbox.low[i];
            if (span >= (1 - EPS) * max_span) {
                float mn = get(vacc[ind], i), mx = mn;
                for (size_t k = 1; k < count; ++k) {
                    const float v = get(vacc[ind + k], i);
                    if (v < mn) mn = v;
                    if (v > mx) mx = v;
                }
                const float spread = mx - mn;
                if (spread > max_spread) { cutfeat = i; max_spread = spread; min_elem = mn; max_elem = mx; }
            }
        }
        const float split_val = (bbox.low[cutfeat] + bbox.high[cutfeat]) / 2;
        if (split_val < min_elem) cutval = min_elem;
        else if (split_val > max_elem) cutval = max_elem;
        else cutval = split_val;
        size_t lim1, lim2;
        plane_split(ind, count, cutfeat, cutval, lim1, lim2);
        if (lim1 > count / 2) index = lim1;
        else if (lim2 < count / 2) index = lim2;
        else index = count / 2;
    }

    void plane_split(size_t ind, size_t count, int cutfeat, float cutval, size_t& lim1, size_t& lim2) {
        size_t left = 0, right = count - 1;
        for (;;) {
            while (left <= right && get(vacc[ind + left], cutfeat) < cutval) ++left;
            while (right && left <= right && get(vacc[ind + right], cutfeat) >= cutval) --right;
            if (left > right || !right) break;
            std::swap(vacc[ind + left], vacc[ind + right]);
            ++left;
            --right;
        }
        lim1 = left;
        right = count - 1;
        for (;;) {
            while (left <= right && get(vacc[ind + left], cutfeat) <= cutval) ++left;
            while (right && left <= right && get(vacc[ind + right], cutfeat) > cutval) --right;
            if (left > right || !right) break;
            std::swap(vacc[ind + left], vacc[ind + right]);
            ++left;
            --right;
        }
        lim2 = left;
    }

    // L2_Simple_Adaptor::evalMetric (:638-649): ((0 + d0^2) + d1^2) + d2^2 in fp32
    float metric(const float q[3], uint32_t i) const {
        float r = 0.0f;
        for (int d = 0; d < 3; ++d) { const float df = q[d] - get(i, d); r += df * df; }
        return r;
    }

    struct Result {                          // KNNResultSet<float, uint32_t>, capacity 5
        uint32_t idx[5];
        float dist[5];
        size_t count = 0;
        float worst() const { return (count < 5 || !count) ? std::numeric_limits<float>::max() : dist[count - 1]; }
        void add(float d, uint32_t index) {
            size_t i;
            for (i = count; i > 0; --i) {
                if (dist[i - 1] > d) {
                    if (i < 5) { dist[i] = dist[i - 1]; idx[i] = idx[i - 1]; }
                } else {
                    break;
                }
            }
            if (i < 5) { dist[i] = d; idx[i] = index; }
            if (count < 5) ++count;
        }
    };

    void search_level(Result& rs, const float q[3], int ni, float mindist, float (&dists)[3]) const {
        const Node& nd = nodes[ni];
        if (nd.child1 < 0 && nd.child2 < 0) {
            const float worst = rs.worst();
            for (size_t i = nd.left; i < nd.right; ++i) {
                const float d = metric(q, vacc[i]);
                if (d < worst) rs.add(d, vacc[i]);
            }
            return;
        }
        const int f = nd.divfeat;
        const float val = q[f];
        const float diff1 = val - nd.divlow, diff2 = val - nd.divhigh;
        int best, other;
        float cut;
        if ((diff1 + diff2) < 0) { best = nd.child1; other = nd.child2; cut = (val - nd.divhigh) * (val - nd.divhigh); }
        else { best = nd.child2; other = nd.child1; cut = (val - nd.divlow) * (val - nd.divlow); }
        search_level(rs, q, best, mindist, dists);
        const float dst = dists[f];
        mindist = mindist + cut - dst;
        dists[f] = cut;
        if (mindist * 1.0f <= rs.worst()) search_level(rs, q, other, mindist, dists);
        dists[f] = dst;
    }

    void knn5(const float q[3], int idx[5], float dist[5], int& found) const {
        found = 0;
        if (root < 0) return;
        float dists[3] = {0.0f, 0.0f, 0.0f};
        float d0 = 0.0f;
        for (int d = 0; d < 3; ++d) {            // computeInitialDistances (:1429-1453)
            if (q[d] < root_bbox.low[d]) { dists[d] = (q[d] - root_bbox.low[d]) * (q[d] - root_bbox.low[d]); d0 += dists[d]; }
            if (q[d] > root_bbox.high[d]) { dists[d] = (q[d] - root_bbox.high[d]) * (q[d] - root_bbox.high[d]); d0 += dists[d]; }
        }
        Result rs;
        search_level(rs, q, root, d0, dists);
        found = static_cast<int>(rs.count);
        for (int k = 0; k < found; ++k) { idx[k] = static_cast<int>(rs.idx[k]); dist[k] = rs.dist[k]; }
    }

    // true when searchLevel reaches original index a before b for query q: descend while both vAcc_ positions
    // fall on the same side of a node's split; at the first node that separates them the near child
    // ((q - divlow) + (q - divhigh) < 0 -> child1) is visited first; inside one leaf, vAcc_ order
    bool visit_before(const float q[3], uint32_t a, uint32_t b) const {
        const size_t pa = vpos[a], pb = vpos[b];
        int ni = root;
        while (nodes[ni].child1 >= 0) {
            const Node& nd = nodes[ni];
            const bool sa = pa >= nd.mid, sb = pb >= nd.mid;
            if (sa != sb) {
                const float val = q[nd.divfeat];
                const bool near2 = !(((val - nd.divlow) + (val - nd.divhigh)) < 0);
                return sa == near2;
            }
            ni = sa ? nd.child2 : nd.child1;
        }
        return pa < pb;
    }

    // exhaustive 5-NN ranked by (fp32 distance, visit order); non-finite distances are never added (dist < FLT_MAX)
    void knn_brute(const float q[3], int idx[5], float dist[5], int& found) const {
        found = 0;
        const size_t m = pts.size() / 3;
        for (size_t i = 0; i < m; ++i) {
            const float d = metric(q, static_cast<uint32_t>(i));
            if (!(d < std::numeric_limits<float>::max())) continue;
            auto before = [&](float da, uint32_t ia, float db, uint32_t ib) {
                return da < db || (da == db && visit_before(q, ia, ib));
            };
            if (found == 5 && !before(d, static_cast<uint32_t>(i), dist[4], static_cast<uint32_t>(idx[4]))) continue;
            int j = found < 5 ? found : 4;
            if (found < 5) ++found;
            while (j > 0 && before(d, static_cast<uint32_t>(i), dist[j - 1], static_cast<uint32_t>(idx[j - 1]))) {
                dist[j] = dist[j - 1];
                idx[j] = idx[j - 1];
                --j;
            }
            dist[j] = d;
            idx[j] = static_cast<int>(i);
        }
    }
};

struct VoxelMap {
    uint64_t revision = 0;                 // bumped by update / apply_transform (kd-tree cache key)
    mutable KdTree3 kd;
    mutable uint64_t kd_rev = ~0ull;
    float voxel_size = 0.5f;
    int factor = 3;
    float planarity_threshold = 0.1f;
    bool compute_surfels = true;
    int init_hit_count = 1;
    DenseMap<L0Node> L0;
    DenseMap<L1Node> L1;
    // container-operation trace (or_map_trace): the insert / erase / clear sequence the reference's UpdateVoxelMap /
    // ApplyTransformAndRehash issue on m_voxels_L0, m_voxels_L1 and the occupied_children sets, replayed on the real
    // ankerl::unordered_dense containers by oracle/ref/map_order_golden.cpp to pin the iteration orders.
    // Records of 7 int32: op, key xyz, child xyz.  op: 1 L0 insert, 2 L0 erase, 3 L1 insert, 4 L1 erase,
    // 5 child insert (key = L1, child), 6 child erase, 7 L0 clear, 8 L1 clear, 9 end of an update call.
    std::vector<int32_t>* trace = nullptr;
    void emit(int op, const VKey& k, const VKey& c = VKey{0, 0, 0}) {
        if (!trace) return;
        const int32_t r[7] = {op, k.x, k.y, k.z, c.x, c.y, c.z};
        trace->insert(trace->end(), r, r + 7);
    }
    void l0_erase(const VKey& k) { if (L0.erase(k)) emit(2, k); }
    void l1_erase(const VKey& k) { if (L1.erase(k)) emit(4, k); }

    // PointToVoxelKey — VoxelMap.cpp:50-58
    VKey key_of(const float p[3], int level) const {
        float scale = voxel_size;
        if (level == 1) scale *= static_cast<float>(factor);
        VKey k;
        k.x = static_cast<int>(std::floor(p[0] / scale));
        k.y = static_cast<int>(std::floor(p[1] / scale));
        k.z = static_cast<int>(std::floor(p[2] / scale));
        return k;
    }
    // GetParentKey — :60-67
    VKey parent_of(const VKey& k) const {
        int f = factor;
        VKey p;
        p.x = k.x >= 0 ? k.x / f : (k.x - (f - 1)) / f;
        p.y = k.y >= 0 ? k.y / f : (k.y - (f - 1)) / f;
        p.z = k.z >= 0 ? k.z / f : (k.z - (f - 1)) / f;
        return p;
    }
    void register_to_parent(const VKey& k) {                                             // :77-80
        const VKey p = parent_of(k);
        if (trace && !L1.find(p)) emit(3, p);
        if (L1[p].children.insert_key(k)) emit(5, p, k);
    }
    void unregister_from_parent(const VKey& k) {                                        // :82-97
        VKey p = parent_of(k);
        L1Node* n = L1.find(p);
        if (!n) return;
        if (n->children.erase(k)) emit(6, p, k);
        if (n->children.size() < 5) n->has_surfel = false;
        if (n->children.empty()) l1_erase(p);
    }
    void add_point(const float p[3]) {                                                    // :99-120
        VKey key = key_of(p, 0);
        bool was_empty = L0.find(key) == nullptr;
        if (was_empty) emit(1, key);
        L0Node& v = L0[key];
        int n = v.point_count;
        if (n == 0) {
            v.c[0] = p[0]; v.c[1] = p[1]; v.c[2] = p[2];
            v.hit_count = init_hit_count;
            v.point_count = 1;
        } else {
            float nf = static_cast<float>(n), n1 = static_cast<float>(n + 1);
            for (int i = 0; i < 3; ++i) v.c[i] = (v.c[i] * nf + p[i]) / n1;
            v.point_count++;
        }
        if (was_empty) register_to_parent(key);
    }
    // surfel PCA shared by UpdateVoxelMap (:187-261) and RecomputeAllSurfels (:304-366)
    // returns planarity; fills normal/centroid
    float fit_surfel(const std::vector<std::array<float, 3>>& cs, float normal[3], float centroid[3]) {
        float c[3] = {0.0f, 0.0f, 0.0f};
        for (auto& p : cs) for (int i = 0; i < 3; ++i) c[i] += p[i];
        float nf = static_cast<float>(cs.size());
        for (int i = 0; i < 3; ++i) c[i] /= nf;
        M3 cov; for (int r = 0; r < 3; ++r) for (int q = 0; q < 3; ++q) cov.a[r][q] = 0.0f;
        for (auto& p : cs) {
            float d[3] = {p[0] - c[0], p[1] - c[1], p[2] - c[2]};
            for (int q = 0; q < 3; ++q) for (int r = 0; r < 3; ++r) cov.a[r][q] += d[q] * d[r];
        }
        for (int r = 0; r < 3; ++r) for (int q = 0; q < 3; ++q) cov.a[r][q] /= nf;
        M3 U, V; float S[3];
        jacobi_svd3(cov, U, S, V);
        for (int i = 0; i < 3; ++i) { normal[i] = U.a[i][2]; centroid[i] = c[i]; }
        return S[2] / (S[0] + 1e-6f);
    }

    void update(const float* xyz, int n, const double sensor[3], double max_distance, bool is_keyframe) {
        update_body(xyz, n, sensor, max_distance, is_keyframe);
        emit(9, VKey{0, 0, 0});
    }
    void update_body(const float* xyz, int n, const double sensor[3], double max_distance, bool is_keyframe) {
        ++revision;
        if (!xyz || n <= 0) return;
        if (!is_keyframe) return;
        float sp[3] = {static_cast<float>(sensor[0]), static_cast<float>(sensor[1]), static_cast<float>(sensor[2])};
        float radius_sq = static_cast<float>(max_distance * max_distance);
        std::vector<VKey> rm;
        for (auto& kv : L0.vals) {
            float d0 = kv.second.c[0] - sp[0], d1 = kv.second.c[1] - sp[1], d2 = kv.second.c[2] - sp[2];
            float dsq = dot3f(d0, d1, d2, d0, d1, d2);
            if (dsq > radius_sq) rm.push_back(kv.first);
        }
        for (auto& k : rm) { unregister_from_parent(k); l0_erase(k); }
        std::vector<VKey> rm1;
        for (auto& kv : L1.vals) if (kv.second.children.empty()) rm1.push_back(kv.first);
        for (auto& k : rm1) l1_erase(k);

        KeySet affected;
        for (int i = 0; i < n; ++i) {
            const float* p = xyz + 3 * i;
            add_point(p);
            affected.insert_key(key_of(p, 1));
        }
        if (!compute_surfels) return;
        const int MIN_CHILDREN = 5;
        for (auto& akv : affected.vals) {
            const VKey key1 = akv.first;
            L1Node* node = L1.find(key1);
            if (!node) continue;
            int cnt = static_cast<int>(node->children.size());
            if (cnt < MIN_CHILDREN) { node->has_surfel = false; continue; }
            if (node->has_surfel && node->last_child_count == cnt) continue;
            std::vector<std::array<float, 3>> cs;
            cs.reserve(cnt);
            for (auto& ck : node->children.vals) {
                const L0Node* l0 = L0.find(ck.first);
                if (l0) cs.push_back({l0->c[0], l0->c[1], l0->c[2]});
            }
            if (cs.size() < 3) { node->has_surfel = false; continue; }
            float nrm[3], cen[3];
            float planarity = fit_surfel(cs, nrm, cen);
            if (planarity > planarity_threshold) {
                node->has_surfel = false;
                std::vector<VKey> kids;
                for (auto& ck : node->children.vals) kids.push_back(ck.first);
                for (auto& k : kids) l0_erase(k);
                l1_erase(key1);
                continue;
            }
            node->has_surfel = true;
            for (int i = 0; i < 3; ++i) { node->normal[i] = nrm[i]; node->centroid[i] = cen[i]; }
            node->planarity = planarity;
            node->last_child_count = cnt;
        }
    }

    void recompute_all_surfels() {   // :304-366
        const int MIN_CHILDREN = 5;
        for (auto& kv : L1.vals) {
            L1Node& node = kv.second;
            int cnt = static_cast<int>(node.children.size());
            if (cnt < MIN_CHILDREN) { node.has_surfel = false; continue; }
            std::vector<std::array<float, 3>> cs;
            for (auto& ck : node.children.vals) {
                const L0Node* l0 = L0.find(ck.first);
                if (l0) cs.push_back({l0->c[0], l0->c[1], l0->c[2]});
            }
            if (cs.size() < static_cast<size_t>(MIN_CHILDREN)) { node.has_surfel = false; continue; }
            float nrm[3], cen[3];
            float planarity = fit_surfel(cs, nrm, cen);
            if (planarity > planarity_threshold) { node.has_surfel = false; continue; }
            node.has_surfel = true;
            for (int i = 0; i < 3; ++i) { node.normal[i] = nrm[i]; node.centroid[i] = cen[i]; }
            node.planarity = planarity;
            node.last_child_count = cnt;
        }
    }

    void apply_transform(const float T[12]) {   // ApplyTransformAndRehash :264-302
        ++revision;
        SE3 s = se3_from12(T);
        std::vector<std::pair<VKey, L0Node>> tr;
        tr.reserve(L0.size());
        for (auto& kv : L0.vals) {
            L0Node nn = kv.second;
            float rc[3]; mul3v(s.R, kv.second.c, rc);
            for (int i = 0; i < 3; ++i) nn.c[i] = rc[i] + s.t[i];
            tr.emplace_back(key_of(nn.c, 0), nn);
        }
        L0.clear(); L1.clear();
        emit(7, VKey{0, 0, 0});
        emit(8, VKey{0, 0, 0});
        for (auto& kn : tr) {
            if (trace && !L0.find(kn.first)) emit(1, kn.first);
            L0Node& ex = L0[kn.first];
            if (ex.point_count == 0) ex = kn.second;
            else {
                float n1 = static_cast<float>(ex.point_count), n2 = static_cast<float>(kn.second.point_count);
                for (int i = 0; i < 3; ++i) ex.c[i] = (ex.c[i] * n1 + kn.second.c[i] * n2) / (n1 + n2);
                ex.point_count += kn.second.point_count;
            }
            register_to_parent(kn.first);
        }
        recompute_all_surfels();
        emit(9, VKey{0, 0, 0});
    }

    // GetSurfelAtPoint — :368-386
    bool lookup(const float p[3], float n[3], float c[3]) const {
        VKey k = key_of(p, 1);
        const L1Node* node = L1.find(k);
        if (!node || !node->has_surfel) return false;
        for (int i = 0; i < 3; ++i) { n[i] = node->normal[i]; c[i] = node->centroid[i]; }
        return true;
    }
};

/* ===================================================================================== */
/*  PKO — AdaptiveMEstimator.cpp                                                          */
/* ===================================================================================== */

struct PKO {
    or_pko_cfg cfg;
    std::vector<double> alphas, Z;
    std::vector<double> w, mu, var;

    double kernel(double r, double delta) const {   // pko_kernel_weight :128-156 (+ :99-126)
        switch (cfg.kernel) {
            case 0: {                                                            // "huber"
                double a = std::fabs(r);
                return a <= delta ? 1.0 : delta / a;
            }
            case 2: {                                                            // tukey_weight :99-108
                double a = std::fabs(r);
                if (a < delta) { double x = a / delta, x2 = x * x; return (1 - x2) * (1 - x2); }
                return 0.0;
            }
            case 3: { double e2 = r * r, d2 = delta * delta; return std::exp(-e2 / d2 / 2.0); }       // :110-114
            case 4: { double e2 = r * r, d2 = delta * delta; return r * d2 / (d2 + e2) / (d2 + e2); } // :116-120
            case 5: { double e = r, d2 = delta * delta; return d2 / std::pow(d2 + e * e, 1.5); }      // :122-126
            default: { double e2 = r * r, d2 = delta * delta; return d2 / (d2 + e2); }               // "cauchy" / other
        }
    }
    double partition(double alpha) const {          // :692-708
        const double bound = cfg.truncated_threshold, step = 0.01;
        double integral = 0.0;
        for (double x = 0.0; x <= bound; x += step) integral += kernel(x, alpha) * step;
        return std::max(integral, 1e-10);
    }
    void init_tables() {                             // initialize_pko :218-241
        int S = cfg.num_alpha_segments;
        alphas.assign(S + 1, 0.0); Z.assign(S + 1, 0.0);
        alphas[0] = cfg.min_scale_factor;
        Z[0] = partition(cfg.min_scale_factor);
        for (int i = 1; i <= S; ++i) {
            double t = static_cast<double>(i) / static_cast<double>(S);
            double ls = (std::pow(100.0, t) - 1.0) / 99.0;
            double a = cfg.min_scale_factor + (cfg.max_scale_factor - cfg.min_scale_factor) * ls;
            alphas[i] = a; Z[i] = partition(a);
        }
    }
    static double gpdf(double x, double mean, double variance) {   // :675-685
        if (variance <= 0.0) return 0.0;
        double diff = x - mean;
        double expo = -0.5 * (diff * diff) / variance;
        double norm = 1.0 / std::sqrt(2.0 * M_PI * variance);
        return norm * std::exp(expo);
    }
    void fit_gmm(const std::vector<double>& res) {   // :294-485
        int n = static_cast<int>(res.size());
        int sample_size = cfg.gmm_sample_size > 0 ? cfg.gmm_sample_size
                                                  : std::min(std::max(100, static_cast<int>(n * 0.1)), 10000);
        if (sample_size > n) sample_size = n;
        std::vector<int> idx(n);
        std::iota(idx.begin(), idx.end(), 0);
        std::mt19937 g(42);
        std::shuffle(idx.begin(), idx.end(), g);
        std::vector<double> sd(sample_size);
        for (int i = 0; i < sample_size; ++i) sd[i] = res[idx[i]];
        n = sample_size;
        const int K = cfg.gmm_components;
        std::mt19937 gen(42);
        std::uniform_int_distribution<> dis(0, static_cast<int>(sd.size()) - 1);
        mu.assign(K, 0.0);
        mu[0] = 0.0;
        for (int i = 1; i < K; ++i) mu[i] = sd[dis(gen)];
        std::vector<int> clusters(sd.size());
        std::vector<double> nm(K);
        while (true) {
            for (size_t i = 0; i < sd.size(); ++i) {
                double md = std::numeric_limits<double>::max();
                int ci = 0;
                for (int j = 0; j < K; ++j) {
                    double d = std::fabs(sd[i] - mu[j]);
                    if (d < md) { md = d; ci = j; }
                }
                clusters[i] = ci;
            }
            std::fill(nm.begin(), nm.end(), 0.0);
            std::vector<int> counts(K, 0);
            for (size_t i = 0; i < sd.size(); ++i) { nm[clusters[i]] += sd[i]; counts[clusters[i]]++; }
            for (int j = 0; j < K; ++j) {
                if (j == 0) nm[j] = 0.0;
                else if (counts[j] > 0) nm[j] /= static_cast<double>(counts[j]);
            }
            if (mu == nm) break;
            nm[0] = 0.0;
            mu = nm;
        }
        double mean = std::accumulate(sd.begin(), sd.end(), 0.0) / sd.size();
        double iv = 0.0;
        for (double x : sd) iv += std::pow(x - mean, 2);
        iv /= sd.size();
        var.assign(K, iv);
        std::vector<int> cc(K, 0);
        for (size_t i = 0; i < sd.size(); ++i) cc[clusters[i]]++;
        w.resize(K);
        for (int j = 0; j < K; ++j) w[j] = static_cast<double>(cc[j]) / static_cast<double>(sd.size());

        std::vector<std::vector<double>> resp(n, std::vector<double>(K));
        for (int it = 0; it < 100; ++it) {
            std::vector<double> sr(n, 0.0);
            for (int i = 0; i < n; ++i) {
                for (int j = 0; j < K; ++j) { resp[i][j] = w[j] * gpdf(sd[i], mu[j], var[j]); sr[i] += resp[i][j]; }
                for (int j = 0; j < K; ++j) resp[i][j] /= sr[i];
            }
            std::vector<double> Nk(K, 0.0);
            for (int j = 0; j < K; ++j) for (int i = 0; i < n; ++i) Nk[j] += resp[i][j];
            std::vector<double> nw(K), nmu(K, 0.0), nv(K, 0.0);
            for (int j = 0; j < K; ++j) {
                nw[j] = Nk[j] / static_cast<double>(n);
                if (j == 0) nmu[j] = 0.0;
                else { for (int i = 0; i < n; ++i) nmu[j] += resp[i][j] * sd[i]; nmu[j] /= Nk[j]; }
                for (int i = 0; i < n; ++i) { double d = sd[i] - nmu[j]; nv[j] += resp[i][j] * d * d; }
                nv[j] /= Nk[j];
                nv[j] = std::max(nv[j], 1e-6);
            }
            double change = 0.0;
            for (int j = 1; j < K; ++j) change += std::fabs(nmu[j] - mu[j]);
            w = nw; nmu[0] = 0.0; mu = nmu; var = nv;
            if (change < 1e-6) break;
        }
    }
    double js(double alpha) const {                 // calculate_js_divergence :710-787
        const int segs = 100;
        double dr = cfg.truncated_threshold / static_cast<double>(segs);
        double pf = 0.0;
        for (size_t j = 0; j < alphas.size(); ++j) if (std::fabs(alphas[j] - alpha) < 1e-10) { pf = Z[j]; break; }
        if (pf == 0.0) pf = partition(alpha);
        if (pf < 1e-10) return std::numeric_limits<double>::max();
        double cost = 0.0, cnt = 0.0;
        for (int i = 0; i < segs; ++i) {
            double r = dr * (1 + static_cast<double>(i));
            double Pr = 0.0;
            if (!w.empty() && !mu.empty() && !var.empty())
                for (int m = 0; m < cfg.gmm_components && m < static_cast<int>(w.size()); ++m) Pr += w[m] * gpdf(r, mu[m], var[m]);
            Pr += 1e-10;
            double kv = kernel(r, alpha);
            double Q = kv / (pf + 1e-10) + 1e-10;
            double M = 0.5 * (Pr + Q);
            double jsd = 0.5 * (Pr * std::log(Pr / M) + Q * std::log(Q / M));
            if (std::isnan(jsd)) continue;
            cost += jsd; cnt += 1.0;
        }
        if (cnt == 0) return std::numeric_limits<double>::max();
        return cost / cnt;
    }
    double scale_factor(const std::vector<double>& res) {   // calculate_scale_factor :63-79 + :243-291
        if (res.empty()) return 1.0;
        if (alphas.empty()) init_tables();
        fit_gmm(res);
        double best_a = cfg.min_scale_factor, best_c = std::numeric_limits<double>::max();
        for (size_t i = 1; i < alphas.size(); ++i) {
            double c = js(alphas[i]);
            if (c < best_c) { best_c = c; best_a = alphas[i]; }
        }
        return best_a;
    }
};

/* ===================================================================================== */
/*  Point cloud utilities                                                                 */
/* ===================================================================================== */

// transform_point_cloud (PointCloudUtils.cpp:102-125): Matrix4f * Vector4f(x,y,z,1), packet order
static inline void transform_pt(const SE3& T, const float p[3], float o[3]) {
    for (int r = 0; r < 3; ++r) {
        float acc = T.R.a[r][0] * p[0];
        acc = T.R.a[r][1] * p[1] + acc;
        acc = T.R.a[r][2] * p[2] + acc;
        acc = T.t[r] * 1.0f + acc;
        o[r] = acc;
    }
}

// FastVoxelFilter::filter (VoxelMap.h:73-104)
struct FilterAcc { float sx = 0.0f, sy = 0.0f, sz = 0.0f; uint32_t count = 0; };
static inline uint64_t expand_bits_filter(uint64_t v) {
    v = v & 0x1FFFFF;
    v = (v | (v << 32)) & 0x1F00000000FFFFULL;
    v = (v | (v << 16)) & 0x1F0000FF0000FFULL;
    v = (v | (v << 8)) & 0x100F00F00F00F00FULL;
    v = (v | (v << 4)) & 0x10C30C30C30C30C3ULL;
    v = (v | (v << 2)) & 0x1249249249249249ULL;
    return v;
}

/* ===================================================================================== */
/*  ICP — IterativeClosestPointOptimizer.cpp                                              */
/* ===================================================================================== */

struct Corr {   // DualFrameCorrespondences (IterativeClosestPointOptimizer.h:128-144)
    std::vector<std::array<double, 3>> last, curr, normals;
    std::vector<double> residuals;
    void clear() { last.clear(); curr.clear(); normals.clear(); residuals.clear(); }
    size_t size() const { return last.size(); }
};

static size_t find_corr(const VoxelMap& map, const float* pts, int n, const SE3& T, double maxd, Corr& c,
                        uint8_t* valid_out, double* res_out) {
    c.clear();
    if (map.L0.empty()) return 0;
    if (n <= 0) return 0;
    std::vector<float> world(static_cast<size_t>(n) * 3);
    for (int i = 0; i < n; ++i) transform_pt(T, pts + 3 * i, &world[3 * i]);
    for (int i = 0; i < n; ++i) {
        const float* q = &world[3 * i];
        if (valid_out) { valid_out[i] = 0; res_out[i] = 0.0; }
        float nf[3], cf[3];
        if (!map.lookup(q, nf, cf)) continue;
        double d0 = static_cast<double>(q[0]) - static_cast<double>(cf[0]);
        double d1 = static_cast<double>(q[1]) - static_cast<double>(cf[1]);
        double d2 = static_cast<double>(q[2]) - static_cast<double>(cf[2]);
        double r = std::fabs(dot3d(nf[0], nf[1], nf[2], d0, d1, d2));
        if (r > maxd) continue;
        c.last.push_back({static_cast<double>(cf[0]), static_cast<double>(cf[1]), static_cast<double>(cf[2])});
        c.curr.push_back({static_cast<double>(pts[3 * i]), static_cast<double>(pts[3 * i + 1]), static_cast<double>(pts[3 * i + 2])});
        c.normals.push_back({static_cast<double>(nf[0]), static_cast<double>(nf[1]), static_cast<double>(nf[2])});
        c.residuals.push_back(r);
        if (valid_out) { valid_out[i] = 1; res_out[i] = r; }
    }
    return c.size();
}

static bool g_kd_use_tree = true;      // or_set_kdtree_search(0) -> exhaustive scan, nanoflann order

/* ---- KDTree variant (find_correspondences_kdtree :647-767): exact 5-NN from the restated nanoflann tree, or
 * (or_set_kdtree_search(0)) the exhaustive scan ranked by the same (distance, visit order) ---- */
// symmetric 3x3 eigen decomposition in double (cyclic Jacobi); returns eigenvector of smallest eigenvalue
// Cyclic Jacobi on the 3x3 scatter matrix.  Stopping rule as Eigen's JacobiSVD (JacobiSVD.h compute(): a pair is
// rotated only while |a_pq| > max(DBL_MIN, 2 eps * maxDiagEntry), the running maximum of the |diagonal|; the sweep
// loop ends after a sweep that rotated nothing): ~4 sweeps on plane-like neighbourhoods instead of the ~11 an
// absolute off-diagonal test down to 1e-300 needs.
static void smallest_eigvec3d(const double A_in[3][3], double v_out[3]) {
    double A[3][3], V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    std::memcpy(A, A_in, sizeof(A));
    double maxd = std::max(std::fabs(A[0][0]), std::max(std::fabs(A[1][1]), std::fabs(A[2][2])));
    for (int sweep = 0; sweep < 50; ++sweep) {
        bool rotated = false;
        for (int p = 0; p < 2; ++p) for (int q = p + 1; q < 3; ++q) {
            const double thr = std::max(std::numeric_limits<double>::min(), 2.0 * std::numeric_limits<double>::epsilon() * maxd);
            if (!(std::fabs(A[p][q]) > thr)) continue;
            rotated = true;
            double theta = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
            double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
            double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
            for (int k = 0; k < 3; ++k) {
                double akp = A[k][p], akq = A[k][q];
                A[k][p] = c * akp - s * akq; A[k][q] = s * akp + c * akq;
            }
            for (int k = 0; k < 3; ++k) {
                double apk = A[p][k], aqk = A[q][k];
                A[p][k] = c * apk - s * aqk; A[q][k] = s * apk + c * aqk;
            }
            for (int k = 0; k < 3; ++k) {
                double vkp = V[k][p], vkq = V[k][q];
                V[k][p] = c * vkp - s * vkq; V[k][q] = s * vkp + c * vkq;
            }
            maxd = std::max(maxd, std::max(std::fabs(A[p][p]), std::fabs(A[q][q])));
        }
        if (!rotated) break;
    }
    int mi = 0;
    for (int i = 1; i < 3; ++i) if (A[i][i] < A[mi][mi]) mi = i;
    for (int k = 0; k < 3; ++k) v_out[k] = V[k][mi];
}

static size_t find_corr_kdtree(const VoxelMap& map, const float* pts, int n, const SE3& T, double maxd, Corr& c,
                               uint8_t* valid_out, double* res_out, float* nout, float* tout) {
    c.clear();
    if (map.L0.empty() || n <= 0) return 0;
    std::vector<float> cloud;   // GetPointCloud (:388-403), L0 iteration order
    cloud.reserve(map.L0.size() * 3);
    for (auto& kv : map.L0.vals) { cloud.push_back(kv.second.c[0]); cloud.push_back(kv.second.c[1]); cloud.push_back(kv.second.c[2]); }
    const bool use_tree = g_kd_use_tree;
    if (map.kd_rev != map.revision) { map.kd.build(cloud); map.kd_rev = map.revision; }   // RebuildKdTree
    for (int i = 0; i < n; ++i) {
        if (valid_out) { valid_out[i] = 0; res_out[i] = 0.0; }
        float q[3]; transform_pt(T, pts + 3 * i, q);
        int idx[5]; float dist[5]; int found;
        if (use_tree) map.kd.knn5(q, idx, dist, found);
        else map.kd.knn_brute(q, idx, dist, found);
        if (found < 5) continue;
        double P[5][3];
        for (int k = 0; k < 5; ++k) for (int d = 0; d < 3; ++d) P[k][d] = cloud[3 * idx[k] + d];
        // is_collinear(p0,p1,p2,0.5) :785-792
        double v1[3], v2[3];
        for (int d = 0; d < 3; ++d) { v1[d] = P[1][d] - P[0][d]; v2[d] = P[2][d] - P[0][d]; }
        double n1 = std::sqrt(dot3d(v1[0], v1[1], v1[2], v1[0], v1[1], v1[2]));
        double n2 = std::sqrt(dot3d(v2[0], v2[1], v2[2], v2[0], v2[1], v2[2]));
        if (n1 > 0) for (int d = 0; d < 3; ++d) v1[d] /= n1;
        if (n2 > 0) for (int d = 0; d < 3; ++d) v2[d] /= n2;
        double cr[3] = {v1[1] * v2[2] - v1[2] * v2[1], v1[2] * v2[0] - v1[0] * v2[2], v1[0] * v2[1] - v1[1] * v2[0]};
        if (std::sqrt(dot3d(cr[0], cr[1], cr[2], cr[0], cr[1], cr[2])) < 0.5) continue;
        double cen[3] = {0, 0, 0};
        for (int k = 0; k < 5; ++k) for (int d = 0; d < 3; ++d) cen[d] += P[k][d];
        for (int d = 0; d < 3; ++d) cen[d] /= 5.0;
        double S[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
        for (int k = 0; k < 5; ++k) {
            double a[3] = {P[k][0] - cen[0], P[k][1] - cen[1], P[k][2] - cen[2]};
            for (int r = 0; r < 3; ++r) for (int s = 0; s < 3; ++s) S[r][s] += a[r] * a[s];
        }
        double nrm[3];
        smallest_eigvec3d(S, nrm);
        double pd = -dot3d(nrm[0], nrm[1], nrm[2], cen[0], cen[1], cen[2]);
        double dist_pl = std::fabs(dot3d(nrm[0], nrm[1], nrm[2], q[0], q[1], q[2]) + pd);
        if (dist_pl > maxd) continue;
        c.last.push_back({cen[0], cen[1], cen[2]});
        c.curr.push_back({static_cast<double>(pts[3 * i]), static_cast<double>(pts[3 * i + 1]), static_cast<double>(pts[3 * i + 2])});
        c.normals.push_back({nrm[0], nrm[1], nrm[2]});
        c.residuals.push_back(dist_pl);
        if (valid_out) { valid_out[i] = 1; res_out[i] = dist_pl; }
        if (nout) for (int d = 0; d < 3; ++d) { nout[3 * i + d] = static_cast<float>(nrm[d]); tout[3 * i + d] = static_cast<float>(cen[d]); }
    }
    return c.size();
}

// Weighted normal equations (:345-410)
static void build_ne(const Corr& c, const SE3& T, const or_icp_cfg& cfg, double scale, double delta_a,
                     float H[6][6], float g[6], float& cost) {
    for (int r = 0; r < 6; ++r) { g[r] = 0.0f; for (int q = 0; q < 6; ++q) H[r][q] = 0.0f; }
    cost = 0.0f;
    const M3& R = T.R;
    const double sden = std::max(scale, 1e-6);
    for (size_t i = 0; i < c.size(); ++i) {
        float p[3], q[3], n[3];
        for (int d = 0; d < 3; ++d) {
            p[d] = static_cast<float>(c.curr[i][d]);
            q[d] = static_cast<float>(c.last[i][d]);
            n[d] = static_cast<float>(c.normals[i][d]);
        }
        float Rp[3]; mul3v(R, p, Rp);
        float pw[3] = {Rp[0] + T.t[0], Rp[1] + T.t[1], Rp[2] + T.t[2]};
        float residual = dot3f(n[0], n[1], n[2], pw[0] - q[0], pw[1] - q[1], pw[2] - q[2]);
        float nres = static_cast<float>(c.residuals[i] / sden);
        float J[6];
        for (int j = 0; j < 3; ++j) J[j] = dot3f(n[0], n[1], n[2], R.a[0][j], R.a[1][j], R.a[2][j]);
        float nn[3] = {-n[0], -n[1], -n[2]};
        float a[3];
        for (int j = 0; j < 3; ++j) a[j] = dot3f(nn[0], nn[1], nn[2], R.a[0][j], R.a[1][j], R.a[2][j]);
        M3 S = hat3(p);
        for (int j = 0; j < 3; ++j) J[3 + j] = dot3f(a[0], a[1], a[2], S.a[0][j], S.a[1][j], S.a[2][j]);
        float w = 1.0f;
        if (cfg.use_robust_loss) {
            float an = std::fabs(nres);
            float dl = static_cast<float>(delta_a);
            if (cfg.loss_cauchy) { float ratio = an / dl; w = 1.0f / (1.0f + ratio * ratio); }
            else if (an > dl) w = dl / an;
        }
        float wJ[6];
        for (int j = 0; j < 6; ++j) wJ[j] = w * J[j];
        for (int col = 0; col < 6; ++col) for (int row = 0; row < 6; ++row) H[row][col] += J[col] * wJ[row];
        float wr = w * residual;
        for (int j = 0; j < 6; ++j) g[j] += wr * J[j];
        cost += wr * residual;
    }
}

static double iter0_scale(const std::vector<double>& res_in) {   // :304-316
    std::vector<double> r = res_in;
    std::sort(r.begin(), r.end());
    double mean = std::accumulate(r.begin(), r.end(), 0.0) / r.size();
    double var = 0.0;
    for (double v : r) var += (v - mean) * (v - mean);
    var /= r.size();
    return std::sqrt(var) / 6.0;
}

// One GN step on a correspondence set (:304-449): iteration-0 scale, PKO delta, normal equations, LDLT, right
// update, log; returns true when |dt| and |dw| are both below tolerance.
static bool gn_step(const Corr& c, SE3& cur, const or_icp_cfg& cfg, PKO& pko, double& scale, int it, or_iter_log* L) {
    if (it == 0 && !c.residuals.empty()) scale = iter0_scale(c.residuals);
    double delta_a = cfg.robust_loss_delta;
    if (cfg.use_pko) {
        std::vector<double> nr;
        nr.reserve(c.residuals.size());
        for (double r : c.residuals) nr.push_back(r / std::max(scale, 1e-6));
        if (!nr.empty()) delta_a = pko.scale_factor(nr);
    }
    float H[6][6], g[6], cost;
    build_ne(c, cur, cfg, scale, delta_a, H, g, cost);
    float Hf[36], mg[6], delta[6];
    for (int r = 0; r < 6; ++r) for (int q = 0; q < 6; ++q) Hf[r * 6 + q] = H[r][q];
    for (int j = 0; j < 6; ++j) mg[j] = -g[j];
    ldlt6_solve(Hf, mg, delta);
    float dt[3] = {delta[0], delta[1], delta[2]}, dw[3] = {delta[3], delta[4], delta[5]};
    SE3 dT;
    if (norm3f(dw) < 1e-10f) dT.R = so3_normalize(eye3());
    else dT.R = so3_exp(dw);
    for (int d = 0; d < 3; ++d) dT.t[d] = dt[d];
    cur = se3_mul(cur, dT);
    float tdel = norm3f(dt), rdel = norm3f(dw);
    if (L) {
        se3_to12(cur, L->pose);
        L->n_corr = static_cast<int>(c.size());
        L->scale = scale;
        L->alpha = delta_a;
        L->cost = cost;
        int k = 0;
        for (int r = 0; r < 6; ++r) for (int q = r; q < 6; ++q) L->H[k++] = H[r][q];
        for (int j = 0; j < 6; ++j) { L->g[j] = g[j]; L->delta[j] = delta[j]; }
    }
    return (tdel < cfg.translation_tolerance) && (rdel < cfg.rotation_tolerance);
}

static int icp_optimize(const VoxelMap& map, const float* pts, int n, const float Ti[12], float To[12],
                        const or_icp_cfg& cfg, bool kdtree, or_iter_log* logs, int* iters_out) {
    SE3 cur = se3_from12(Ti);
    std::memcpy(To, Ti, sizeof(float) * 12);
    PKO pko; pko.cfg = cfg.pko;
    double scale = 1.0;
    int iters = 0;
    Corr c;
    for (int it = 0; it < cfg.max_iterations; ++it) {
        size_t nc = kdtree ? find_corr_kdtree(map, pts, n, cur, cfg.max_correspondence_distance, c, nullptr, nullptr, nullptr, nullptr)
                           : find_corr(map, pts, n, cur, cfg.max_correspondence_distance, c, nullptr, nullptr);
        if (nc < static_cast<size_t>(cfg.min_correspondence_points)) {
            if (iters_out) *iters_out = iters;
            return 0;
        }
        const bool conv = gn_step(c, cur, cfg, pko, scale, it, logs ? &logs[it] : nullptr);
        ++iters;
        if (conv) break;
    }
    se3_to12(cur, To);
    if (iters_out) *iters_out = iters;
    return 1;
}

/* ---- loop-closure ICP: optimize_loop (:40-251) + find_correspondences_loop (:465-585) ----
 * Query = curr point through the curr pose (Matrix4f * Vector4f, :500-503); exact 5-NN in the matched keyframe's
 * local map (its feature cloud through its pose, :60-64); the collinearity gate and plane fit of the KDTree path;
 * NO distance gate (:573); target = neighbour 0 in the matched frame, T_lw * p in fp64 (:517-520), cast to fp32
 * and put back in the world, R_m q + t_m (:148-150).  T_lw is the rigid inverse [R^T | -R^T t] in fp64 rounded to
 * fp32; the reference's Matrix4f::inverse() agrees with it to fp32 rounding (parity unpinned at that level; the
 * target only enters H and g).  Up to 100 iterations; success = converged AND inlier ratio >= 0.5. */
static size_t find_corr_loop(const KdTree3& kd, const std::vector<float>& lmap, const float* pts, int n, const SE3& T,
                             const float Tlw[12], const SE3& Tm, Corr& c) {
    c.clear();
    if (n <= 0 || lmap.empty()) return 0;
    for (int i = 0; i < n; ++i) {
        float q[3]; transform_pt(T, pts + 3 * i, q);
        int idx[5]; float dist[5]; int found;
        if (g_kd_use_tree) kd.knn5(q, idx, dist, found);
        else kd.knn_brute(q, idx, dist, found);
        if (found < 5) continue;
        double P[5][3];
        for (int k = 0; k < 5; ++k) for (int d = 0; d < 3; ++d) P[k][d] = lmap[3 * idx[k] + d];
        double v1[3], v2[3];
        for (int d = 0; d < 3; ++d) { v1[d] = P[1][d] - P[0][d]; v2[d] = P[2][d] - P[0][d]; }
        double n1 = std::sqrt(dot3d(v1[0], v1[1], v1[2], v1[0], v1[1], v1[2]));
        double n2 = std::sqrt(dot3d(v2[0], v2[1], v2[2], v2[0], v2[1], v2[2]));
        if (n1 > 0) for (int d = 0; d < 3; ++d) v1[d] /= n1;
        if (n2 > 0) for (int d = 0; d < 3; ++d) v2[d] /= n2;
        double cr[3] = {v1[1] * v2[2] - v1[2] * v2[1], v1[2] * v2[0] - v1[0] * v2[2], v1[0] * v2[1] - v1[1] * v2[0]};
        if (std::sqrt(dot3d(cr[0], cr[1], cr[2], cr[0], cr[1], cr[2])) < 0.5) continue;   // is_collinear (:785-792)
        double cen[3] = {0, 0, 0};
        for (int k = 0; k < 5; ++k) for (int d = 0; d < 3; ++d) cen[d] += P[k][d];
        for (int d = 0; d < 3; ++d) cen[d] /= 5.0;
        double S[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
        for (int k = 0; k < 5; ++k) {
            double a[3] = {P[k][0] - cen[0], P[k][1] - cen[1], P[k][2] - cen[2]};
            for (int r = 0; r < 3; ++r) for (int s2 = 0; s2 < 3; ++s2) S[r][s2] += a[r] * a[s2];
        }
        double nrm[3];
        smallest_eigvec3d(S, nrm);
        double pd = -dot3d(nrm[0], nrm[1], nrm[2], cen[0], cen[1], cen[2]);
        double dist_pl = std::fabs(dot3d(nrm[0], nrm[1], nrm[2], q[0], q[1], q[2]) + pd);
        float lf[3], qw[3];
        for (int r = 0; r < 3; ++r)
            lf[r] = static_cast<float>(((static_cast<double>(Tlw[4 * r]) * P[0][0] + static_cast<double>(Tlw[4 * r + 1]) * P[0][1]) +
                                        static_cast<double>(Tlw[4 * r + 2]) * P[0][2]) + static_cast<double>(Tlw[4 * r + 3]));
        for (int r = 0; r < 3; ++r) qw[r] = dot3f(Tm.R.a[r][0], Tm.R.a[r][1], Tm.R.a[r][2], lf[0], lf[1], lf[2]) + Tm.t[r];
        // the world target goes where find_corr_kdtree keeps the centroid: build_ne reads it as q
        c.last.push_back({static_cast<double>(qw[0]), static_cast<double>(qw[1]), static_cast<double>(qw[2])});
        c.curr.push_back({static_cast<double>(pts[3 * i]), static_cast<double>(pts[3 * i + 1]), static_cast<double>(pts[3 * i + 2])});
        c.normals.push_back({nrm[0], nrm[1], nrm[2]});
        c.residuals.push_back(dist_pl);
    }
    return c.size();
}

static int icp_optimize_loop(const float* curr, int ncur, const float Tc[12], const float* matched, int nm,
                             const float Tmat[12], const or_icp_cfg& cfg, float Trel[12], float* inlier,
                             or_iter_log* logs, int max_logs, int* iters_out, int* conv_out) {
    SE3 cur = se3_from12(Tc);
    const SE3 Tm = se3_from12(Tmat);
    PKO pko; pko.cfg = cfg.pko;                 // m_adaptive_estimator->reset() (:53-55): no state survives anyway
    std::vector<float> lmap(3 * static_cast<size_t>(std::max(nm, 0)));
    for (int i = 0; i < nm; ++i) transform_pt(Tm, matched + 3 * i, &lmap[3 * i]);
    KdTree3 kd;
    kd.build(lmap);
    float Tlw[12];
    for (int r = 0; r < 3; ++r) {
        double tr = 0.0;
        for (int k = 0; k < 3; ++k) {
            Tlw[4 * r + k] = Tmat[4 * k + r];
            tr -= static_cast<double>(Tmat[4 * k + r]) * static_cast<double>(Tmat[4 * k + 3]);
        }
        Tlw[4 * r + 3] = static_cast<float>(tr);
    }
    double scale = 1.0;
    int iters = 0;
    bool converged = false;
    Corr c;
    for (int it = 0; it < 100; ++it) {
        const size_t nc = find_corr_loop(kd, lmap, curr, ncur, cur, Tlw, Tm, c);
        if (nc < static_cast<size_t>(cfg.min_correspondence_points)) break;
        const bool conv = gn_step(c, cur, cfg, pko, scale, it, (logs && it < max_logs) ? &logs[it] : nullptr);
        ++iters;
        if (conv) { converged = true; break; }
    }
    if (iters_out) *iters_out = iters;
    if (conv_out) *conv_out = converged ? 1 : 0;
    if (!converged) return 0;
    // optimized_relative_transform = curr.pose.Inverse() * optimized_curr_pose (:240)
    SE3 ci = se3_from12(Tc), inv;
    M3 Rt;
    for (int r = 0; r < 3; ++r) for (int k = 0; k < 3; ++k) Rt.a[r][k] = ci.R.a[k][r];
    inv.R = so3_normalize(Rt);
    const float mt[3] = {-ci.t[0], -ci.t[1], -ci.t[2]};
    mul3v(inv.R, mt, inv.t);
    se3_to12(se3_mul(inv, cur), Trel);
    // inlier ratio (:206-238): t + R p, nearest matched point by nanoflann's fp32 squared L2, sqrt < 1
    int inl = 0;
    for (int i = 0; i < ncur; ++i) {
        const float* p = curr + 3 * i;
        float w[3];
        for (int r = 0; r < 3; ++r) w[r] = cur.t[r] + dot3f(cur.R.a[r][0], cur.R.a[r][1], cur.R.a[r][2], p[0], p[1], p[2]);
        float best = FLT_MAX;
        bool any = false;
        for (int k = 0; k < nm; ++k) {
            const float d0 = w[0] - lmap[3 * k], d1 = w[1] - lmap[3 * k + 1], d2 = w[2] - lmap[3 * k + 2];
            const float d = (d0 * d0 + d1 * d1) + d2 * d2;
            if (d < best) { best = d; any = true; }
        }
        if (any && std::sqrt(best) < 1.0f) ++inl;
    }
    *inlier = static_cast<float>(inl) / static_cast<float>(ncur);
    return *inlier < 0.5f ? 0 : 1;
}

}  // namespace orc

using namespace orc;

/* ===================================================================================== */
/*  C ABI                                                                                 */
/* ===================================================================================== */

extern "C" {

double or_pko_scale_factor(const or_pko_cfg* cfg, const double* residuals, int n, double* gmm_out) {
    PKO p; p.cfg = *cfg;
    std::vector<double> r(residuals, residuals + n);
    double a = p.scale_factor(r);
    if (gmm_out && n > 0) {
        int K = cfg->gmm_components;
        for (int j = 0; j < K; ++j) { gmm_out[j] = p.w[j]; gmm_out[K + j] = p.mu[j]; gmm_out[2 * K + j] = p.var[j]; }
    }
    return a;
}

void or_shuffle_prefix(int n, int k, int* out) {
    std::vector<int> idx(n);
    std::iota(idx.begin(), idx.end(), 0);
    std::mt19937 g(42);
    std::shuffle(idx.begin(), idx.end(), g);
    for (int i = 0; i < k && i < n; ++i) out[i] = idx[i];
}

void or_kmeans_seed_draws(int m, int count, int* out) {
    std::mt19937 gen(42);
    std::uniform_int_distribution<> dis(0, m - 1);
    for (int i = 0; i < count; ++i) out[i] = dis(gen);
}

void or_pko_tables(const or_pko_cfg* cfg, double* alphas, double* Z) {
    PKO p; p.cfg = *cfg;
    p.init_tables();
    for (size_t i = 0; i < p.alphas.size(); ++i) { alphas[i] = p.alphas[i]; Z[i] = p.Z[i]; }
}

// SE3::Inverse (MathUtils.h:155-158): SO3(R^T), R_inv * (-t)
void or_se3_inverse(const float A[12], float out[12]) {
    SE3 a = se3_from12(A), o;
    M3 Rt;
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) Rt.a[r][c] = a.R.a[c][r];
    o.R = so3_normalize(Rt);
    const float mt[3] = {-a.t[0], -a.t[1], -a.t[2]};
    mul3v(o.R, mt, o.t);
    se3_to12(o, out);
}

// should_create_keyframe's two measures (Estimator.cpp:349-368): |t - t_kf| and |SO3::Log(R_kf^-1 R)|
// (SO3::Log, MathUtils.cpp:41-84; SO3 inverse and product both re-project through SO3(Matrix3f))
void or_keyframe_metrics(const float kf[12], const float pose[12], double out[2]) {
    SE3 K = se3_from12(kf), P = se3_from12(pose);
    const float d[3] = {P.t[0] - K.t[0], P.t[1] - K.t[1], P.t[2] - K.t[2]};
    out[0] = norm3f(d);
    M3 Kt;
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) Kt.a[r][c] = K.R.a[c][r];
    const M3 m = so3_normalize(mul33(so3_normalize(Kt), P.R));
    const float tr = (m.a[0][0] + m.a[1][1]) + m.a[2][2];
    const float ct = (tr - 1.0f) * 0.5f;
    const float th = std::acos(std::max(-1.0f, std::min(1.0f, ct)));
    float w[3];
    if (th < 1e-6f) {
        w[0] = m.a[2][1] - 0.0f; w[1] = m.a[0][2] - 0.0f; w[2] = m.a[1][0] - 0.0f;
    } else {
        const float st = std::sin(th);
        if (std::fabs(st) < 1e-6f) {
            int mi = 0;
            if (m.a[1][1] > m.a[0][0]) mi = 1;
            if (m.a[2][2] > m.a[mi][mi]) mi = 2;
            float ax[3];
            ax[mi] = std::sqrt((m.a[mi][mi] + 1.0f) * 0.5f);
            for (int i = 0; i < 3; ++i) if (i != mi) ax[i] = m.a[mi][i] / (2.0f * ax[mi]);
            const float sk[3] = {(m.a[2][1] - m.a[1][2]) * 0.5f, (m.a[0][2] - m.a[2][0]) * 0.5f, (m.a[1][0] - m.a[0][1]) * 0.5f};
            if (dot3f(ax[0], ax[1], ax[2], sk[0], sk[1], sk[2]) < 0) for (float& a : ax) a = -a;
            for (int i = 0; i < 3; ++i) w[i] = ax[i] * th;
        } else {
            const float f = th / (2.0f * st);
            w[0] = f * (m.a[2][1] - m.a[1][2]); w[1] = f * (m.a[0][2] - m.a[2][0]); w[2] = f * (m.a[1][0] - m.a[0][1]);
        }
    }
    out[1] = norm3f(w);
}

void or_se3_compose(const float A[12], const float B[12], float out[12]) {
    se3_to12(se3_mul(se3_from12(A), se3_from12(B)), out);
}
void or_so3_exp(const float w[3], float R[9]) {
    M3 m = so3_exp(w);
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) R[r * 3 + c] = m.a[r][c];
}
void or_so3_normalize(const float Rin[9], float Rout[9]) {
    M3 m; for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) m.a[r][c] = Rin[r * 3 + c];
    M3 o = so3_normalize(m);
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) Rout[r * 3 + c] = o.a[r][c];
}
int or_jacobi_svd3(const float A[9], float U[9], float S[3], float V[9]) {
    M3 a; for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) a.a[r][c] = A[r * 3 + c];
    M3 u, v;
    int rc = jacobi_svd3(a, u, S, v);
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) { U[r * 3 + c] = u.a[r][c]; V[r * 3 + c] = v.a[r][c]; }
    return rc;
}
void or_ldlt6_solve(const float H[36], const float b[6], float x[6]) { ldlt6_solve(H, b, x); }

void* or_map_create(float voxel_size, int hierarchy_factor, float planarity_threshold, int compute_surfels) {
    VoxelMap* m = new VoxelMap();
    m->voxel_size = voxel_size;
    m->factor = hierarchy_factor;
    m->planarity_threshold = planarity_threshold;
    m->compute_surfels = compute_surfels != 0;
    return m;
}
void or_map_destroy(void* m) { VoxelMap* v = static_cast<VoxelMap*>(m); delete v->trace; delete v; }
void or_map_update(void* m, const float* xyz, int n, const double sensor[3], double max_distance, int is_keyframe) {
    static_cast<VoxelMap*>(m)->update(xyz, n, sensor, max_distance, is_keyframe != 0);
}
void or_map_apply_transform(void* m, const float T[12]) { static_cast<VoxelMap*>(m)->apply_transform(T); }

void or_map_trace(void* m, int enable) {
    VoxelMap* vm = static_cast<VoxelMap*>(m);
    delete vm->trace;
    vm->trace = enable ? new std::vector<int32_t>() : nullptr;
}

size_t or_map_trace_get(const void* m, int32_t* out, size_t cap) {
    const VoxelMap* vm = static_cast<const VoxelMap*>(m);
    if (!vm->trace) return 0;
    const size_t n = vm->trace->size();
    if (out) std::memcpy(out, vm->trace->data(), std::min(n, cap) * sizeof(int32_t));
    return n;
}

// Iteration orders: L0 keys, L1 keys, and each L1's children (concatenated, L1 order) -- int32 xyz triples.
size_t or_map_orders(const void* m, int32_t* l0, int32_t* l1, int32_t* child_cnt, int32_t* children, size_t cap) {
    const VoxelMap* vm = static_cast<const VoxelMap*>(m);
    size_t nc = 0;
    for (auto& kv : vm->L1.vals) nc += kv.second.children.size();
    if (!l0) return nc;
    size_t i = 0;
    for (auto& kv : vm->L0.vals) { l0[3 * i] = kv.first.x; l0[3 * i + 1] = kv.first.y; l0[3 * i + 2] = kv.first.z; ++i; }
    i = 0;
    size_t c = 0;
    for (auto& kv : vm->L1.vals) {
        l1[3 * i] = kv.first.x; l1[3 * i + 1] = kv.first.y; l1[3 * i + 2] = kv.first.z;
        child_cnt[i] = static_cast<int32_t>(kv.second.children.size());
        for (auto& ck : kv.second.children.vals) {
            if (c < cap) { children[3 * c] = ck.first.x; children[3 * c + 1] = ck.first.y; children[3 * c + 2] = ck.first.z; }
            ++c;
        }
        ++i;
    }
    return nc;
}
int or_map_l0_count(void* m) { return static_cast<int>(static_cast<VoxelMap*>(m)->L0.size()); }
int or_map_l1_count(void* m) { return static_cast<int>(static_cast<VoxelMap*>(m)->L1.size()); }
int or_map_surfel_count(void* m) {
    int c = 0;
    for (auto& kv : static_cast<VoxelMap*>(m)->L1.vals) if (kv.second.has_surfel) ++c;
    return c;
}
int or_map_get_surfels(void* m, int32_t* keys, float* normals, float* centroids, float* planarity, int cap) {
    int c = 0;
    for (auto& kv : static_cast<VoxelMap*>(m)->L1.vals) {
        if (!kv.second.has_surfel) continue;
        if (c >= cap) break;
        keys[3 * c] = kv.first.x; keys[3 * c + 1] = kv.first.y; keys[3 * c + 2] = kv.first.z;
        for (int i = 0; i < 3; ++i) { normals[3 * c + i] = kv.second.normal[i]; centroids[3 * c + i] = kv.second.centroid[i]; }
        if (planarity) planarity[c] = kv.second.planarity;
        ++c;
    }
    return c;
}
int or_map_get_l0(void* m, float* xyz, int cap) {
    int c = 0;
    for (auto& kv : static_cast<VoxelMap*>(m)->L0.vals) {
        if (c >= cap) break;
        for (int i = 0; i < 3; ++i) xyz[3 * c + i] = kv.second.c[i];
        ++c;
    }
    return c;
}
int or_map_lookup(void* m, const float p[3], float n[3], float c[3]) { return static_cast<VoxelMap*>(m)->lookup(p, n, c) ? 1 : 0; }

int or_voxel_filter(const float* in, int n, float voxel_size, int stride, float* out) {
    if (n <= 0 || stride < 1) return 0;
    const float inv = 1.0f / voxel_size;
    std::vector<uint64_t> keys_order;
    struct KV { uint64_t k; FilterAcc a; };
    std::vector<KV> vals;
    std::vector<uint32_t> buckets(1024, 0u);
    uint64_t mask = 1023;
    auto hk = [](uint64_t k) { __uint128_t r = static_cast<__uint128_t>(k) * 0x9E3779B97F4A7C15ULL; return static_cast<uint64_t>(r) ^ static_cast<uint64_t>(r >> 64); };
    for (int i = 0; i < n; i += stride) {
        const float* p = in + 3 * i;
        if (!std::isfinite(p[0]) || !std::isfinite(p[1]) || !std::isfinite(p[2])) continue;
        const int64_t OFF = (1 << 20);
        int64_t ix = static_cast<int64_t>(std::floor(p[0] * inv)) + OFF;
        int64_t iy = static_cast<int64_t>(std::floor(p[1] * inv)) + OFF;
        int64_t iz = static_cast<int64_t>(std::floor(p[2] * inv)) + OFF;
        ix = std::max<int64_t>(0, std::min<int64_t>(ix, (1 << 21) - 1));
        iy = std::max<int64_t>(0, std::min<int64_t>(iy, (1 << 21) - 1));
        iz = std::max<int64_t>(0, std::min<int64_t>(iz, (1 << 21) - 1));
        uint64_t key = expand_bits_filter(static_cast<uint64_t>(ix)) | (expand_bits_filter(static_cast<uint64_t>(iy)) << 1) |
                       (expand_bits_filter(static_cast<uint64_t>(iz)) << 2);
        uint64_t b = hk(key) & mask;
        int64_t vi = -1;
        while (buckets[b]) { if (vals[buckets[b] - 1].k == key) { vi = buckets[b] - 1; break; } b = (b + 1) & mask; }
        if (vi < 0) {
            vals.push_back({key, FilterAcc()});
            vi = static_cast<int64_t>(vals.size() - 1);
            buckets[b] = static_cast<uint32_t>(vi + 1);
            if (vals.size() * 5 > buckets.size() * 4) {
                buckets.assign(buckets.size() * 2, 0u); mask = buckets.size() - 1;
                for (size_t j = 0; j < vals.size(); ++j) { uint64_t bb = hk(vals[j].k) & mask; while (buckets[bb]) bb = (bb + 1) & mask; buckets[bb] = static_cast<uint32_t>(j + 1); }
            }
        }
        FilterAcc& a = vals[vi].a;
        a.sx += p[0]; a.sy += p[1]; a.sz += p[2]; a.count++;
    }
    int c = 0;
    for (auto& kv : vals) {
        float ic = 1.0f / static_cast<float>(kv.a.count);
        out[3 * c] = kv.a.sx * ic; out[3 * c + 1] = kv.a.sy * ic; out[3 * c + 2] = kv.a.sz * ic;
        ++c;
    }
    return c;
}

void or_transform_points(const float* in, int n, const float T[12], float* out) {
    SE3 s = se3_from12(T);
    for (int i = 0; i < n; ++i) transform_pt(s, in + 3 * i, out + 3 * i);
}

int or_find_correspondences(void* map, const float* pts, int n, const float T[12], double maxd, uint8_t* valid, double* residual) {
    Corr c;
    return static_cast<int>(find_corr(*static_cast<VoxelMap*>(map), pts, n, se3_from12(T), maxd, c, valid, residual));
}

void or_set_kdtree_search(int use_tree) { g_kd_use_tree = use_tree != 0; }

void or_kdtree_knn5(const float* cloud, int m, const float* q, int nq, int use_tree, int* idx, float* dist, int* found) {
    KdTree3 kd;
    kd.build(std::vector<float>(cloud, cloud + 3 * static_cast<size_t>(std::max(m, 0))));
    for (int i = 0; i < nq; ++i) {
        int* ix = idx + 5 * static_cast<size_t>(i);
        float* ds = dist + 5 * static_cast<size_t>(i);
        for (int k = 0; k < 5; ++k) { ix[k] = -1; ds[k] = std::numeric_limits<float>::infinity(); }
        if (use_tree) kd.knn5(q + 3 * static_cast<size_t>(i), ix, ds, found[i]);
        else kd.knn_brute(q + 3 * static_cast<size_t>(i), ix, ds, found[i]);
    }
}

int or_find_correspondences_kdtree(void* map, const float* pts, int n, const float T[12], double maxd, uint8_t* valid,
                                   double* residual, float* normal_out, float* target_out) {
    Corr c;
    return static_cast<int>(find_corr_kdtree(*static_cast<VoxelMap*>(map), pts, n, se3_from12(T), maxd, c, valid, residual,
                                             normal_out, target_out));
}

int or_icp_optimize(void* map, const float* pts, int n, const float T_init[12], float T_out[12], const or_icp_cfg* cfg,
                    int use_kdtree, or_iter_log* logs, int* iterations) {
    return icp_optimize(*static_cast<VoxelMap*>(map), pts, n, T_init, T_out, *cfg, use_kdtree != 0, logs, iterations);
}

int or_icp_optimize_loop(const float* curr, int n_curr, const float T_curr[12], const float* matched, int n_matched,
                         const float T_matched[12], const or_icp_cfg* cfg, float T_rel[12], float* inlier_ratio,
                         or_iter_log* logs, int max_logs, int* iterations, int* converged) {
    return icp_optimize_loop(curr, n_curr, T_curr, matched, n_matched, T_matched, *cfg, T_rel, inlier_ratio, logs,
                             max_logs, iterations, converged);
}

int or_build_normal_equations(void* map, const float* pts, int n, const float T[12], const or_icp_cfg* cfg, double scale,
                              double delta, float H[36], float g[6], float* cost) {
    Corr c;
    SE3 s = se3_from12(T);
    size_t nc = find_corr(*static_cast<VoxelMap*>(map), pts, n, s, cfg->max_correspondence_distance, c, nullptr, nullptr);
    float Hm[6][6];
    build_ne(c, s, *cfg, scale, delta, Hm, g, *cost);
    for (int r = 0; r < 6; ++r) for (int q = 0; q < 6; ++q) H[r * 6 + q] = Hm[r][q];
    return static_cast<int>(nc);
}

}  // extern "C"
