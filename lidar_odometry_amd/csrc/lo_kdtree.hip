// lo_kdtree.hip — KDTree correspondence variant (use_surfel_correspondence = false) on the device.
//
// Reference: IterativeClosestPointOptimizer::find_correspondences_kdtree (IterativeClosestPointOptimizer.cpp:
// 647-767), is_collinear (:785-792), KdTree::nearestKSearch (PointCloudUtils.h:398-423) over nanoflann 1.7.1
// (L2_Simple_Adaptor, KNNResultSet; thirdparty/nanoflann/nanoflann.hpp:199-282, :1885-1905) built on the
// map's L0 centroids (VoxelMap::GetPointCloud :388-403, RebuildKdTree :420-438).
//
// The kd-tree is an ordering device; what the reference consumes is the exact 5-NN set by fp32 squared L2
// distance ((0 + dx^2) + dy^2) + dz^2, sorted ascending.  MI355X-first, the search runs on a dense uniform
// grid over the centroids (built on the host at map upload, lo_map_set_points), 8 lanes per query:
//   k_knn        shells of cells around the query cell, rows split over the query's lanes (batched loads,
//                butterfly merge of per-lane top-5 lists); after shell r the result is certified once the 5th
//                distance is below the distance from the query to the scanned cube (minus a margin that
//                covers fp32 binning); otherwise the query goes to
//   k_knn_brute  one workgroup per unresolved query: lane-strided brute force + LDS tree merge of top-5 lists;
//   k_plane      collinearity gate, 5-point centroid / covariance, smallest eigenvector (fp64 cyclic Jacobi,
//                the oracle's restatement of JacobiSVD<MatrixXd>(5x3).matrixV().col(2)), point-to-plane
//                distance <= max_correspondence_distance; writes the per-point plane (fp32-rounded normal and
//                centroid, as .cast<float>() at :361-365), the fp64 distance (residuals[i]) and the same ballots /
//                block statistics as the surfel path, so k_pko_t / k_accumulate run unchanged.
// Equal distances are ranked as nanoflann ranks them: by the order its searchLevel visits the points (an earlier
// visit wins, NANOFLANN_FIRST_MATCH is not defined), evaluated on the reference's own tree (lo_kdorder.h, built with
// the grid) only when two distances are equal -- so the 5-NN lists, their order and their tie-breaks equal
// nanoflann's (tests/test_gpu_kdtree.py against tests/golden/knn_golden.npz, written by nanoflann itself).
// Non-finite queries find nothing (nanoflann only adds points with dist < worstDist = FLT_MAX).
#include "lo_blocksort.h"
#include "lo_device.h"
#include "lo_solve.h"

#include <cfloat>

namespace lo {

constexpr int kKnnRMax = 5;            // grid shells before a query falls back to brute force
constexpr double kKnnMargin = 1e-2;    // m: covers fp32 binning of centroids near cell faces

struct Top5 {
    float d[5];
    int id[5];      // original centroid index (tie-break)
    int pos[5];     // position in kd_pts
    int n;
    float tie;      // fast order only: the smallest distance at which two different points compared equal (+inf:
                    // none); the result can differ from nanoflann's only if tie <= the final fifth distance
};

// The query and the reference tree's order, for ties.
struct KnnQ {
    float q[3];
    const uint32_t* vpos;
    const KdNode* nodes;
};

// nanoflann visits original index a before b (both in the tree): descend while both vAcc_ positions fall on the
// same side of a node's split; the node that separates them is entered on the query's side first
// (searchLevel: (q - divlow) + (q - divhigh) < 0 -> child1, fp32 as nanoflann); one leaf: vAcc_ order.
__device__ __forceinline__ bool kd_visit_before(const KnnQ& Q, int a, int b) {
    const uint32_t pa = Q.vpos[a], pb = Q.vpos[b];
    int ni = 0;
    for (int depth = 0; depth < 64; ++depth) {
        const KdNode nd = Q.nodes[ni];
        if (nd.child1 < 0) break;
        const bool sa = pa >= nd.mid, sb = pb >= nd.mid;
        if (sa != sb) {
            const float val = Q.q[nd.divfeat];
            const bool near2 = !(((val - nd.divlow) + (val - nd.divhigh)) < 0.0f);
            return sa == near2;
        }
        ni = sa ? nd.child2 : nd.child1;
    }
    return pa < pb;
}

// Two orders over (distance, point).  EX: nanoflann's (distance, visit order) -- the reference's result.  Fast:
// (distance, index), which differs only between points at EQUAL distance, and every such comparison raises
// t.tie; a query that raised it is answered again in the exact order (k_knn hands it to k_knn_brute, which reruns
// it with EX), so the visit-order walk stays out of the hot loops.
template <bool EX>
__device__ __forceinline__ bool lex_less(const KnnQ& Q, Top5& t, float da, int ia, float db, int ib) {
    if constexpr (EX) {
        return da < db || (da == db && ia != ib && kd_visit_before(Q, ia, ib));
    } else {
        if (da == db && ia != ib) t.tie = fminf(t.tie, da);
        return da < db || (da == db && ia < ib);
    }
}

__device__ __forceinline__ void top5_init(Top5& t) {
#pragma unroll
    for (int k = 0; k < 5; ++k) { t.d[k] = __builtin_inff(); t.id[k] = 0x7fffffff; t.pos[k] = -1; }
    t.n = 0;
    t.tie = __builtin_inff();
}

// KNNResultSet::addPoint behind searchLevel's `dist < worstDist` (worstDist = FLT_MAX until 5 are held),
// with (dist, visit order) order; unrolled compare-swaps keep the list in VGPRs.
template <bool EX>
__device__ __forceinline__ void top5_insert(const KnnQ& Q, Top5& t, float d, int id, int pos) {
    if (t.n < 5) {
        if (!(d < FLT_MAX)) return;
        ++t.n;
    } else if (!lex_less<EX>(Q, t, d, id, t.d[4], t.id[4])) {
        return;
    }
    t.d[4] = d; t.id[4] = id; t.pos[4] = pos;
#pragma unroll
    for (int k = 4; k > 0; --k) {
        if (lex_less<EX>(Q, t, t.d[k], t.id[k], t.d[k - 1], t.id[k - 1])) {
            const float fd = t.d[k]; t.d[k] = t.d[k - 1]; t.d[k - 1] = fd;
            const int fi = t.id[k]; t.id[k] = t.id[k - 1]; t.id[k - 1] = fi;
            const int fp = t.pos[k]; t.pos[k] = t.pos[k - 1]; t.pos[k - 1] = fp;
        }
    }
}

__device__ __forceinline__ float l2sq(float qx, float qy, float qz, const float4& v) {
    const float dx = qx - v.x, dy = qy - v.y, dz = qz - v.z;
    return (dx * dx + dy * dy) + dz * dz;
}

// Merge of disjoint top-5 lists across the kKnnGroup = 16 lanes of a query: a hypercube over the 16-lane DPP row
// (quad_perm xor 1, quad_perm xor 2, row_half_mirror i <-> 7-i, row_mirror i <-> 15-i) -- VALU moves, no LDS
// round trips -- after which every lane of the row holds the (dist, index)-smallest five of the group's union.
template <int CTRL, bool EX>
__device__ __forceinline__ void top5_merge_dpp(const KnnQ& Q, Top5& t) {
    Top5 u;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        u.d[k] = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(t.d[k]), CTRL, 0xf, 0xf, false));
        u.id[k] = __builtin_amdgcn_mov_dpp(t.id[k], CTRL, 0xf, 0xf, false);
        u.pos[k] = __builtin_amdgcn_mov_dpp(t.pos[k], CTRL, 0xf, 0xf, false);
    }
    u.n = __builtin_amdgcn_mov_dpp(t.n, CTRL, 0xf, 0xf, false);
    t.tie = fminf(t.tie, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(t.tie), CTRL, 0xf, 0xf, false)));
#pragma unroll
    for (int k = 0; k < 5; ++k)
        if (k < u.n) top5_insert<EX>(Q, t, u.d[k], u.id[k], u.pos[k]);
}

template <bool EX>
__device__ __forceinline__ Top5 group_merge(const KnnQ& Q, const Top5& own) {
    static_assert(kKnnGroup == 16, "the DPP hypercube spans one 16-lane row");
    Top5 t = own;
    top5_merge_dpp<0xB1, EX>(Q, t);     // quad_perm [1,0,3,2]
    top5_merge_dpp<0x4E, EX>(Q, t);     // quad_perm [2,3,0,1]
    top5_merge_dpp<0x141, EX>(Q, t);    // row_half_mirror
    top5_merge_dpp<0x140, EX>(Q, t);    // row_mirror
    return t;
}

// ====================================================================================================
// k_knn: grid shells.  kd_nbr[5i] = positions of the 5-NN, -1 = fewer than 5 (rejected), -2 = unresolved
// ====================================================================================================
// One candidate range of the kd_pts array (a run of cells of one grid row), scanned with 8 loads in flight.
// thr: an upper bound on the query's fifth distance (seed_bound), or +inf: a point farther than it can neither be one
// of the five nor tie with the fifth, so it skips the insert.
__device__ __forceinline__ void scan_range8(const KParams& P, const KnnQ& Q, uint32_t s, uint32_t e, float qx, float qy,
                                            float qz, float thr, Top5& t) {
    for (uint32_t p = s; p < e; p += 8) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = (p + u < e) ? P.kd_pts[p + u] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const float d = l2sq(qx, qy, qz, v[u]);
            if (p + u < e && d <= thr) top5_insert<false>(Q, t, d, __float_as_int(v[u].w), static_cast<int>(p + u));
        }
    }
}

// The query's five neighbours of the previous GN iteration (kd_nbr, positions into kd_pts) are five distinct points
// of the set, so the largest of their distances at the new pose bounds the fifth distance from above.  Any five
// distinct positions would do (a stale record of an earlier call too); anything else gives +inf (no bound).
__device__ __forceinline__ float seed_bound(const KParams& P, int i, float qx, float qy, float qz) {
    const int32_t* prev = P.kd_nbr + 5 * static_cast<size_t>(i);
    int pv[5];
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        pv[k] = prev[k];
        ok = ok && pv[k] >= 0 && pv[k] < P.kd_m;
    }
#pragma unroll
    for (int a = 0; a < 5; ++a)
#pragma unroll
        for (int b = a + 1; b < 5; ++b) ok = ok && pv[a] != pv[b];
    if (!ok) return __builtin_inff();
    float s5 = 0.0f;
#pragma unroll
    for (int k = 0; k < 5; ++k) s5 = fmaxf(s5, l2sq(qx, qy, qz, P.kd_pts[pv[k]]));
    return s5;
}

constexpr int kKnnRowsMax = 4;          // rows of one round per lane: r = 3 has 49 rows over 16 lanes

__device__ __forceinline__ void knn_body(const KParams& P, const float (&T)[12], bool seed) {
    // kKnnGroup consecutive lanes (one DPP row) share one query: lane g takes rows g, g + 16, ... of each round.
    // The first round scans the whole 3x3x3 cube (the r = 0 cell alone almost never certifies: its faces are
    // < h / 2 away while the 5th neighbour of a surface sample is ~h); later rounds scan the shell r.  A lane's
    // cell-range bounds for the round are loaded together, then its ranges are scanned 8 points at a time.
    const int gi = blockIdx.x * kBlock + threadIdx.x;
    const int i = gi / kKnnGroup, g = gi % kKnnGroup;
    if (i >= scan_n(P)) return;                              // whole groups leave together
    int32_t* out = P.kd_nbr + 5 * static_cast<size_t>(i);
    float qx, qy, qz;
    transform_pt(T, P.pts[3 * i], P.pts[3 * i + 1], P.pts[3 * i + 2], qx, qy, qz);
    if (!(isfinite(qx) && isfinite(qy) && isfinite(qz)) || P.kd_m < 5) { if (g == 0) out[0] = -1; return; }
    const float h = P.kd_h;
    const float fx = floorf(qx / h), fy = floorf(qy / h), fz = floorf(qz / h);
    if (!(fabsf(fx) < 1e9f && fabsf(fy) < 1e9f && fabsf(fz) < 1e9f)) {
        if (g == 0) { out[0] = -2; P.kd_unres[atomicAdd(&P.st->kd_unres_n, 1u)] = i; }
        return;
    }
    const int c[3] = {static_cast<int>(fx), static_cast<int>(fy), static_cast<int>(fz)};
    const int dimx = P.kd_dim[0], dimy = P.kd_dim[1], dimz = P.kd_dim[2];
    const int ox = P.kd_org[0], oy = P.kd_org[1], oz = P.kd_org[2];
    const double q[3] = {qx, qy, qz};
    const KnnQ Q{{qx, qy, qz}, P.kd_vpos, P.kd_nodes};
    // this lane's rows of round r from j0 on (kKnnRowsMax of them): their range bounds (up to 2 per row: a full row,
    // or the shell's two end cells), loaded together
    auto ranges = [&](int r, int j0, uint32_t (&rs)[2 * kKnnRowsMax], uint32_t (&re)[2 * kKnnRowsMax]) {
        const int side = 2 * r + 1;
#pragma unroll
        for (int j = 0; j < kKnnRowsMax; ++j) {
            rs[2 * j] = re[2 * j] = rs[2 * j + 1] = re[2 * j + 1] = 0;
            const int k = j0 + g + j * kKnnGroup;
            if (k >= side * side) continue;
            const int dz = k / side - r, dy = k % side - r;
            const int z = c[2] + dz - oz, y = c[1] + dy - oy;
            if (z < 0 || z >= dimz || y < 0 || y >= dimy) continue;
            const size_t row = (static_cast<size_t>(z) * dimy + y) * dimx;
            if (r == 1 || dz == -r || dz == r || dy == -r || dy == r) {        // whole row of the cube / shell
                const int x0 = max(c[0] - r - ox, 0), x1 = min(c[0] + r - ox, dimx - 1);
                if (x0 <= x1) { rs[2 * j] = P.kd_start[row + x0]; re[2 * j] = P.kd_start[row + x1 + 1]; }
            } else {                                                            // the two end cells
                const int xa = c[0] - r - ox, xb = c[0] + r - ox;
                if (xa >= 0 && xa < dimx) { rs[2 * j] = P.kd_start[row + xa]; re[2 * j] = P.kd_start[row + xa + 1]; }
                if (xb >= 0 && xb < dimx) { rs[2 * j + 1] = P.kd_start[row + xb]; re[2 * j + 1] = P.kd_start[row + xb + 1]; }
            }
        }
    };
    const float thr = seed ? seed_bound(P, i, qx, qy, qz) : __builtin_inff();   // read before g == 0 rewrites it
    Top5 own, grp;
    top5_init(own);
    bool done = false;
    for (int r = 1; r <= kKnnRMax && !done; ++r) {
        const int side = 2 * r + 1;
        for (int j0 = 0; j0 < side * side; j0 += kKnnRowsMax * kKnnGroup) {
            uint32_t rs[2 * kKnnRowsMax], re[2 * kKnnRowsMax];
            ranges(r, j0, rs, re);
#pragma unroll
            for (int j = 0; j < 2 * kKnnRowsMax; ++j) scan_range8(P, Q, rs[j], re[j], qx, qy, qz, thr, own);
        }
        grp = group_merge<false>(Q, own);
        // every unscanned centroid lies outside the cube of cells [c - r, c + r]
        bool all = true;
        double b = DBL_MAX;
        const int org[3] = {ox, oy, oz}, dim[3] = {dimx, dimy, dimz};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            all = all && (c[a] - r <= org[a]) && (c[a] + r >= org[a] + dim[a] - 1);
            b = fmin(b, q[a] - static_cast<double>(c[a] - r) * h);
            b = fmin(b, static_cast<double>(c[a] + r + 1) * h - q[a]);
        }
        if (all) {
            done = true;
        } else if (grp.n == 5) {
            const double e = b - kKnnMargin;
            done = e > 0.0 && static_cast<double>(grp.d[4]) < e * e * (1.0 - 1e-6);
        }
    }
    if (g != 0) return;
    if (!done || (grp.n == 5 && grp.tie <= grp.d[4]) || (grp.n < 5 && grp.tie < __builtin_inff())) {
        // not certified, or a tie that can decide the five or their order
        out[0] = -2;
        P.kd_unres[atomicAdd(&P.st->kd_unres_n, 1u)] = i;
        return;
    }
    if (grp.n < 5) { out[0] = -1; return; }
#pragma unroll
    for (int k = 0; k < 5; ++k) out[k] = grp.pos[k];
}

__global__ __launch_bounds__(kBlock) void k_knn(KParams P) {
    if (!P.init && P.st->done) return;
    float T[12];
    scan_pose(P, P.init, blockIdx.x, T);
    knn_body(P, T, !P.init);
}

// The solve of GN iteration it fused with the kNN search of iteration it + 1 (small scans with PKO; the
// counterpart of k_solve_correspond in lo_kernels.hip): every block reduces the selected candidate's partials and
// solves redundantly (the same pose everywhere), block 0 publishes the GN state -- k_knn_brute and k_plane read
// the pose from it -- and the old pose comes from the previous iteration's log (the initial pose for it = 0).
__global__ __launch_bounds__(kBlock) void k_solve_knn(KParams P, int it) {
    DevState* st = P.st;
    const int done = st->done;
    const int tid = threadIdx.x, blk = blockIdx.x;
    __shared__ int s_c, s_done, s_skip;
    __shared__ double tot[kNE];
    __shared__ float s_T[12];
    int bi = 0;
    if (tid < kWave) bi = pko_select_index(P);
    if (tid == 0) {                              // thread 0's view of the flag decides for the whole block (block 0
        s_skip = done;                           // of this launch may set it while other blocks start)
        if (!done) {
            s_c = bi > 0 ? bi - 1 : P.NA;
            if (blk == 0) st->alpha = bi > 0 ? P.alphas[bi] : P.min_scale;
        }
    }
    __syncthreads();
    if (s_skip) return;
    solve_sums<kBlock>(P.acc_part + static_cast<size_t>(s_c) * kFuseMaxBlocks * kNE, P.nb_acc, tot);
    if (tid == 0) {
        const float* pose_old = it == 0 ? P.T0 : st->logs[it - 1].pose;
        s_done = solve_core(P, it, tot, pose_old, s_T, blk == 0) ? 1 : 0;
    }
    __syncthreads();
    if (s_done) return;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = s_T[k];
    knn_body(P, T, true);
}

// The KDTree counterpart of k_pick_correspond (reference-exact mode): the record of the candidate the PKO launch
// selected (its reference-order sums and fp32 solve, acc_candidate_exact) is iteration it's pose, block 0 publishes
// it, and every block searches its queries' five neighbours at that pose for iteration it + 1.
__global__ __launch_bounds__(kBlock) void k_pick_knn(KParams P, int it) {
    __shared__ float s_rec[kCandWords];
    bool conv = false;
    if (!pick_select(P, it, s_rec, &conv) || conv) return;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = s_rec[k];
    knn_body(P, T, true);
}

// ====================================================================================================
// k_knn_brute: unresolved queries, one 1024-thread workgroup each (grid-strided over the device-side list):
// every lane scans a strided share of the map with 8 loads in flight, the 64 lanes of a wave merge with a
// hypercube (DPP within 16-lane rows, then __shfl_xor 16 / 32), the 16 wave results meet in LDS and wave 0's
// first row merges them the same way.
// ====================================================================================================
constexpr int kBruteThreads = 1024;

template <bool EX>
__device__ __forceinline__ void top5_merge_xor(const KnnQ& Q, Top5& t, int o) {
    Top5 u;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        u.d[k] = __shfl_xor(t.d[k], o, 64);
        u.id[k] = __shfl_xor(t.id[k], o, 64);
        u.pos[k] = __shfl_xor(t.pos[k], o, 64);
    }
    u.n = __shfl_xor(t.n, o, 64);
    t.tie = fminf(t.tie, __shfl_xor(t.tie, o, 64));
#pragma unroll
    for (int k = 0; k < 5; ++k)
        if (k < u.n) top5_insert<EX>(Q, t, u.d[k], u.id[k], u.pos[k]);
}

// One query over the whole map by a 1024-thread workgroup: every lane scans a strided share with 8 loads in flight,
// then the wave / workgroup merges; wave 0 lane 0 returns the five (and, fast order, whether any tie was seen).
template <bool EX>
__device__ __forceinline__ Top5 brute_query(const KParams& P, const KnnQ& Q, float (&s_d)[16][5], int (&s_id)[16][5],
                                            int (&s_pos)[16][5], int (&s_n)[16], float (&s_tie)[16]) {
    constexpr int kBT = 1024;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const float qx = Q.q[0], qy = Q.q[1], qz = Q.q[2];
    Top5 t;
    top5_init(t);
    for (int p0 = tid; p0 < P.kd_m; p0 += 8 * kBT) {           // 8 loads in flight per lane
        float4 v[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            const int p = p0 + w * kBT;
            v[w] = p < P.kd_m ? P.kd_pts[p] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            const int p = p0 + w * kBT;
            if (p < P.kd_m) top5_insert<EX>(Q, t, l2sq(qx, qy, qz, v[w]), __float_as_int(v[w].w), p);
        }
    }
    t = group_merge<EX>(Q, t);                             // 16-lane rows
    top5_merge_xor<EX>(Q, t, 16);
    top5_merge_xor<EX>(Q, t, 32);                          // the wave's five
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 5; ++k) { s_d[wid][k] = t.d[k]; s_id[wid][k] = t.id[k]; s_pos[wid][k] = t.pos[k]; }
        s_n[wid] = t.n;
        s_tie[wid] = t.tie;
    }
    __syncthreads();
    Top5 a;
    top5_init(a);
    if (wid == 0 && lane < 16) {
#pragma unroll
        for (int k = 0; k < 5; ++k) { a.d[k] = s_d[lane][k]; a.id[k] = s_id[lane][k]; a.pos[k] = s_pos[lane][k]; }
        a.n = s_n[lane];
        a.tie = s_tie[lane];
    }
    if (wid == 0) a = group_merge<EX>(Q, a);               // lanes 16-63 merge empty lists (discarded)
    __syncthreads();
    return a;
}

// A deciding tie met by the fast order (a.n == 5, a.tie <= a.d[4]): the five in nanoflann's order.  The fifth distance
// d5 does not depend on how ties are ranked, so the five are among the points within d5; the workgroup lists them in
// LDS and one lane ranks them by (distance, visit order) -- the only place the visit-order walk is inlined, so the
// kernel needs no call frame (no scratch memory: an empty launch costs what any empty launch costs).  A list longer
// than kExCap (points equidistant by the thousand) is ranked by that lane over the whole set instead.
constexpr int kExCap = 1024;
__device__ __forceinline__ Top5 brute_query_ex(const KParams& P, const KnnQ& Q, float d5, float (&s_ed)[kExCap],
                                               int (&s_ei)[kExCap], int (&s_ep)[kExCap], int& s_en) {
    const int tid = threadIdx.x;
    if (tid == 0) s_en = 0;
    __syncthreads();
    for (int p = tid; p < P.kd_m; p += kBruteThreads) {
        const float4 v = P.kd_pts[p];
        const float d = l2sq(Q.q[0], Q.q[1], Q.q[2], v);
        if (d <= d5) {
            const int k = atomicAdd(&s_en, 1);
            if (k < kExCap) { s_ed[k] = d; s_ei[k] = __float_as_int(v.w); s_ep[k] = p; }
        }
    }
    __syncthreads();
    Top5 t;
    top5_init(t);
    if (tid == 0) {
        const int ne = s_en;
        if (ne <= kExCap) {
            for (int k = 0; k < ne; ++k) top5_insert<true>(Q, t, s_ed[k], s_ei[k], s_ep[k]);
        } else {
            for (int p = 0; p < P.kd_m; ++p) {
                const float4 v = P.kd_pts[p];
                top5_insert<true>(Q, t, l2sq(Q.q[0], Q.q[1], Q.q[2], v), __float_as_int(v.w), p);
            }
        }
    }
    __syncthreads();
    return t;
}

__global__ __launch_bounds__(kBruteThreads) void k_knn_brute(KParams P) {
    DevState* st = P.st;
    if (st->done) return;
    const unsigned nu = st->kd_unres_n;
    if (blockIdx.x >= nu) return;
    constexpr int kW = kBruteThreads / 64;
    __shared__ float s_d[kW][5];
    __shared__ int s_id[kW][5];
    __shared__ int s_pos[kW][5];
    __shared__ int s_n[kW];
    __shared__ float s_tie[kW];
    __shared__ int s_redo, s_five;
    __shared__ float s_d5;
    __shared__ float s_ed[kExCap];
    __shared__ int s_ei[kExCap], s_ep[kExCap], s_en;
    const int tid = threadIdx.x;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
    for (unsigned u = blockIdx.x; u < nu; u += gridDim.x) {
        const int i = P.kd_unres[u];
        float qx, qy, qz;
        transform_pt(T, P.pts[3 * i], P.pts[3 * i + 1], P.pts[3 * i + 2], qx, qy, qz);
        const KnnQ Q{{qx, qy, qz}, P.kd_vpos, P.kd_nodes};
        Top5 a = brute_query<false>(P, Q, s_d, s_id, s_pos, s_n, s_tie);
        if (tid == 0) {                                    // (a is thread 0's: the workgroup's five)
            s_redo = (a.n == 5 && a.tie <= a.d[4]) || (a.n < 5 && a.tie < __builtin_inff());
            s_five = a.n == 5;
            s_d5 = a.d[4];
        }
        __syncthreads();
        const bool redo = s_redo != 0, five = s_five != 0;
        const float d5 = s_d5;
        __syncthreads();
        if (redo) {                                        // a deciding tie: nanoflann's visit order ranks it
            if (P.kd_nodes) {
                // fewer than five: no five to rank (the answer is -1 whatever the order)
                if (five) a = brute_query_ex(P, Q, d5, s_ed, s_ei, s_ep, s_en);   // uniform: every thread calls
            } else if (tid == 0) {
                atomicOr(&st->kd_tie, 1u);                 // no visit order built: the host reruns with it
            }
        }
        if (tid == 0) {
            int32_t* out = P.kd_nbr + 5 * static_cast<size_t>(i);
            if (a.n < 5) out[0] = -1;
            else for (int k = 0; k < 5; ++k) out[k] = a.pos[k];
        }
    }
}

// k_knn_brute_w: the same answers by one wave per unresolved query, for a grid of at most 16k points built without the
// kd visit order (the loop-closure ICP's matched keyframe cloud, a device-built map grid): no LDS, no barrier and no
// call into the visit-order walk (whose call frame puts k_knn_brute on scratch memory), so a launch with nothing to do
// costs what an empty launch costs, and a few dozen queries run side by side.  A deciding tie is ranked by index and
// flagged (DevState::kd_tie) for the host's rerun with the order, as k_knn_brute does without one.
__global__ __launch_bounds__(kBlock) void k_knn_brute_w(KParams P) {
    DevState* st = P.st;
    if (st->done) return;
    const unsigned nu = st->kd_unres_n;
    constexpr int kWpb = kBlock / kWave;
    const int lane = threadIdx.x & 63;
    const unsigned w0 = blockIdx.x * kWpb + (threadIdx.x >> 6);
    if (w0 >= nu) return;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
    const KnnQ Q0{{0.0f, 0.0f, 0.0f}, nullptr, nullptr};
    for (unsigned u = w0; u < nu; u += gridDim.x * kWpb) {
        const int i = P.kd_unres[u];
        float qx, qy, qz;
        transform_pt(T, P.pts[3 * i], P.pts[3 * i + 1], P.pts[3 * i + 2], qx, qy, qz);
        Top5 t;
        top5_init(t);
        for (int p0 = lane; p0 < P.kd_m; p0 += 8 * kWave) {
            float4 v[8];
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                const int p = p0 + w * kWave;
                v[w] = p < P.kd_m ? P.kd_pts[p] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                const int p = p0 + w * kWave;
                if (p < P.kd_m) top5_insert<false>(Q0, t, l2sq(qx, qy, qz, v[w]), __float_as_int(v[w].w), p);
            }
        }
        t = group_merge<false>(Q0, t);
        top5_merge_xor<false>(Q0, t, 16);
        top5_merge_xor<false>(Q0, t, 32);
        if (lane == 0) {
            if ((t.n == 5 && t.tie <= t.d[4]) || (t.n < 5 && t.tie < __builtin_inff())) atomicOr(&st->kd_tie, 1u);
            int32_t* out = P.kd_nbr + 5 * static_cast<size_t>(i);
            if (t.n < 5) out[0] = -1;
            else for (int k = 0; k < 5; ++k) out[k] = t.pos[k];
        }
    }
}

// ====================================================================================================
// Small point sets (the loop-closure ICP's matched keyframe cloud, <= kKnnAllMax points): every query against the
// whole set, staged once per workgroup in LDS (index order, the original index in w).  One wave per query, 16
// queries per 1024-thread workgroup (one LDS copy of the set per 16 queries, 4 waves per SIMD to hide the LDS and
// VALU latency): lane l takes points l, l + 64, ... (a wave reads 64 consecutive points per ds_read_b128), keeps
// its own top-5 list, and the wave merges the 64 lists (DPP rows, then across rows) -- the exact answer by
// construction, no cells, no certification and no brute-force pass.  Fast order (distance, index) as k_knn; a
// query whose five or their order rest on an equal distance is marked -3, k_plane flags it (DevState::kd_tie) and
// the host reruns the solve on the grid with the kd visit order.
// ====================================================================================================
// The set in LDS, padded to a multiple of kAllBatch points with sentinels at +inf (their distance to any finite query
// is +inf: never one of the five, never within 1 m), so the search loops read 8 points per lane with no bounds test.
constexpr int kAllBatch = 8 * kWave;
__device__ __forceinline__ int all_padded(int m) { return (m + kAllBatch - 1) / kAllBatch * kAllBatch; }
__device__ __forceinline__ void stage_all(const KParams& P, float4* s_map) {
    const int m = P.kd_m, mp = all_padded(m);
    const float inf = __builtin_inff();
#pragma unroll 4
    for (int p = threadIdx.x; p < mp; p += kAllThreads) {
        const float4 v = P.kd_pts[min(p, m - 1)];          // in bounds (m >= 1 when the set is searched)
        s_map[p] = p < m ? v : make_float4(inf, inf, inf, __int_as_float(-1));
    }
    __syncthreads();
}

__device__ __forceinline__ float wave_min(float f) {
    f = fminf(f, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(f), 0xB1, 0xf, 0xf, false)));
    f = fminf(f, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(f), 0x4E, 0xf, 0xf, false)));
    f = fminf(f, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(f), 0x141, 0xf, 0xf, false)));
    f = fminf(f, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(f), 0x140, 0xf, 0xf, false)));
    f = fminf(f, __shfl_xor(f, 16, 64));
    return fminf(f, __shfl_xor(f, 32, 64));
}

// seed (GN iterations after the first): the query's five neighbours of the previous iteration are five points of the
// set, so the largest of their distances at the new pose bounds the fifth distance from above -- thr starts there and
// only the few points within it reach the insert (without a seed, thr is the wave's smallest fifth distance so far).
__device__ __forceinline__ void knn_all_body(const KParams& P, const float (&T)[12], const float4* s_map, bool seed) {
    const int i = blockIdx.x * (kAllThreads / kWave) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (i >= scan_n(P)) return;                              // whole waves leave together
    int32_t* out = P.kd_nbr + 5 * static_cast<size_t>(i);
    float qx, qy, qz;
    transform_pt(T, P.pts[3 * i], P.pts[3 * i + 1], P.pts[3 * i + 2], qx, qy, qz);
    if (!(isfinite(qx) && isfinite(qy) && isfinite(qz)) || P.kd_m < 5) { if (lane == 0) out[0] = -1; return; }
    const KnnQ Q{{qx, qy, qz}, nullptr, nullptr};
    const int mp = all_padded(P.kd_m);
    Top5 t;
    top5_init(t);
    // thr: the smallest fifth distance over the wave's lanes so far -- every lane's five are points of the set, so the
    // set's own fifth distance is <= thr, and a point farther than thr can neither be one of the five nor tie with
    // the fifth: only points within thr reach the (branchy) insert, the rest cost a distance and a compare
    float thr = __builtin_inff();
    if (seed) {
        const int32_t* prev = P.kd_nbr + 5 * static_cast<size_t>(i);     // read before lane 0 rewrites it below
        int pv[5];
        bool ok = true;                                      // five distinct points of the set (else no seed)
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            pv[k] = prev[k];
            ok = ok && pv[k] >= 0 && pv[k] < P.kd_m;
        }
#pragma unroll
        for (int a = 0; a < 5; ++a)
#pragma unroll
            for (int b = a + 1; b < 5; ++b) ok = ok && pv[a] != pv[b];
        if (ok) {
            float s5 = 0.0f;
#pragma unroll
            for (int k = 0; k < 5; ++k) s5 = fmaxf(s5, l2sq(qx, qy, qz, s_map[pv[k]]));
            thr = s5;
        }
    }
    if (!(thr < __builtin_inff())) {
        // no seed: a first pass takes each lane's nearest point; the fifth smallest of the 64 lane minima is the
        // distance of five distinct points of the set, so it bounds the fifth distance from above (and equals it
        // whenever the five nearest fall in five different lanes)
        float mn = __builtin_inff();
        for (int p0 = lane; p0 < mp; p0 += kAllBatch) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = s_map[p0 + u * kWave];
#pragma unroll
            for (int u = 0; u < 8; ++u) mn = fminf(mn, l2sq(qx, qy, qz, v[u]));
        }
        for (int r = 0; r < 5; ++r) {                        // remove the wave minimum five times
            thr = wave_min(mn);
            const uint64_t b = __ballot(mn == thr);
            if (b && lane == __builtin_ctzll(b)) mn = __builtin_inff();
        }
    }
    for (int p0 = lane; p0 < mp; p0 += kAllBatch) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = s_map[p0 + u * kWave];
        float d[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) d[u] = l2sq(qx, qy, qz, v[u]);
#if defined(LO_ALL_EXP) && LO_ALL_EXP == 1                 // diagnostic (scripts/knn_microbench): no inserts
        if (p0 == lane) for (int u = 0; u < 5; ++u) top5_insert<false>(Q, t, d[u], p0 + u * kWave, p0 + u * kWave);
        thr = fminf(thr, d[7]);
#else
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (d[u] <= thr) top5_insert<false>(Q, t, d[u], p0 + u * kWave, p0 + u * kWave);
        thr = fminf(thr, wave_min(t.n == 5 ? t.d[4] : __builtin_inff()));
#endif
    }
#if !(defined(LO_ALL_EXP) && LO_ALL_EXP == 2)                // diagnostic: no merges
    t = group_merge<false>(Q, t);                            // 16-lane rows
    top5_merge_xor<false>(Q, t, 16);
    top5_merge_xor<false>(Q, t, 32);                         // the wave's five
#endif
    if (lane != 0) return;
    if ((t.n == 5 && t.tie <= t.d[4]) || (t.n < 5 && t.tie < __builtin_inff())) { out[0] = -3; return; }
    if (t.n < 5) { out[0] = -1; return; }
#pragma unroll
    for (int k = 0; k < 5; ++k) out[k] = t.pos[k];
}

__global__ __launch_bounds__(kAllThreads) void k_knn_all(KParams P) {
    extern __shared__ float4 s_map[];
    if (!P.init && P.st->done) return;
    float T[12];
    scan_pose(P, P.init, blockIdx.x, T);
    stage_all(P, s_map);
    knn_all_body(P, T, s_map, !P.init);
}

// k_pick_knn over a small set
__global__ __launch_bounds__(kAllThreads) void k_pick_knn_all(KParams P, int it) {
    extern __shared__ float4 s_map[];
    __shared__ float s_rec[kCandWords];
    bool conv = false;
    if (!pick_select(P, it, s_rec, &conv) || conv) return;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = s_rec[k];
    stage_all(P, s_map);
    knn_all_body(P, T, s_map, true);
}

// k_inlier over a small set, a wave per point: its lanes take every 64th point until one lies within 1 m (an existence
// test, so the order of the scan does not matter).  std::sqrt(sqdist) < 1.0f (:233) is sqdist < 1.0f: a correctly
// rounded square root is monotone and exact at 1, and the largest float below 1 has its root rounded below 1.
__global__ __launch_bounds__(kAllThreads) void k_inlier_all(KParams P) {
    extern __shared__ float4 s_map[];
    __shared__ unsigned s_hits[kAllThreads / kWave];
    DevState* st = P.st;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
    stage_all(P, s_map);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * (kAllThreads / kWave) + wid;
    bool in = false;
    if (i < scan_n(P)) {
        const float px = P.pts[3 * i], py = P.pts[3 * i + 1], pz = P.pts[3 * i + 2];
        const float q[3] = {T[3] + dot3f(T[0], T[1], T[2], px, py, pz), T[7] + dot3f(T[4], T[5], T[6], px, py, pz),
                            T[11] + dot3f(T[8], T[9], T[10], px, py, pz)};
        if (isfinite(q[0]) && isfinite(q[1]) && isfinite(q[2]) && P.kd_m > 0) {
            const int mp = all_padded(P.kd_m);
            for (int p0 = lane; p0 < mp; p0 += kAllBatch) {          // 8 LDS reads in flight
                float4 v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = s_map[p0 + u * kWave];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const float d0 = q[0] - v[u].x, d1 = q[1] - v[u].y, d2 = q[2] - v[u].z;
                    in = in || (d0 * d0 + d1 * d1) + d2 * d2 < 1.0f;
                }
                if (__ballot(in)) break;                             // the wave found one
            }
        }
    }
    const bool hit = __ballot(in) != 0;
    if (lane == 0) s_hits[wid] = hit ? 1u : 0u;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned h = 0;
        for (int w = 0; w < kAllThreads / kWave; ++w) h += s_hits[w];
        if (h) atomicAdd(&st->inliers, h);
    }
}

// lo_knn_search (kNN without the plane stage): the unresolved-query counter k_plane would zero
__global__ void k_knn_reset(KParams P) {
    if (threadIdx.x == 0) P.st->kd_unres_n = 0;
}

// ====================================================================================================
// k_plane: plane fit + residual + the correspondence epilogue
// ====================================================================================================
__device__ __forceinline__ double dot3d(double a0, double a1, double a2, double b0, double b1, double b2) {
    const double e0 = a0 * b0, e1 = a1 * b1, e2 = a2 * b2;       // Vector3d dot: (e0 + e1) + e2
    return (e0 + e1) + e2;
}

// Smallest-eigenvalue eigenvector of a symmetric 3x3 (cyclic Jacobi, fp64) -- the same sweep and stopping rule as the
// oracle's smallest_eigvec3d (oracle/src/lo_oracle.cpp; Eigen JacobiSVD's: rotate a pair only while
// |a_pq| > max(DBL_MIN, 2 eps * running max |diagonal|), stop after a sweep without rotations), so normals agree bit
// for bit under -ffp-contract=off.  Fully unrolled (p, q) rotations keep A and V in registers.
__device__ __forceinline__ bool jrot(double (&A)[3][3], double (&V)[3][3], int p, int q, double& maxd) {
    const double thr = std_max(DBL_MIN, 2.0 * DBL_EPSILON * maxd);     // std::max semantics, as the oracle
    if (!(fabs(A[p][q]) > thr)) return false;
    const double theta = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
    const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
    const double cc = 1.0 / sqrt(t * t + 1.0), s = t * cc;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double akp = A[k][p], akq = A[k][q];
        A[k][p] = cc * akp - s * akq; A[k][q] = s * akp + cc * akq;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double apk = A[p][k], aqk = A[q][k];
        A[p][k] = cc * apk - s * aqk; A[q][k] = s * apk + cc * aqk;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double vkp = V[k][p], vkq = V[k][q];
        V[k][p] = cc * vkp - s * vkq; V[k][q] = s * vkp + cc * vkq;
    }
    maxd = std_max(maxd, std_max(fabs(A[p][p]), fabs(A[q][q])));
    return true;
}

__device__ __forceinline__ void smallest_eigvec3d(double (&A)[3][3], double (&v)[3]) {
    double V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    double maxd = std_max(fabs(A[0][0]), std_max(fabs(A[1][1]), fabs(A[2][2])));
    for (int sweep = 0; sweep < 50; ++sweep) {
        bool rot = jrot(A, V, 0, 1, maxd);
        rot = jrot(A, V, 0, 2, maxd) || rot;
        rot = jrot(A, V, 1, 2, maxd) || rot;
        if (!rot) break;
    }
    int mi = 0;
    if (A[1][1] < A[0][0]) mi = 1;
    if (A[2][2] < (mi == 0 ? A[0][0] : A[1][1])) mi = 2;
#pragma unroll
    for (int k = 0; k < 3; ++k) v[k] = (mi == 0) ? V[k][0] : (mi == 1 ? V[k][1] : V[k][2]);
}

__global__ __launch_bounds__(kBlock) void k_plane(KParams P, int with_stats) {
    DevState* st = P.st;
    if (st->done) return;
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x == 0) {                        // k_knn_brute has drained the list
        st->dbg[15] = st->kd_unres_n;                                 // last unresolved count (lo_debug_counters)
        st->kd_unres_n = 0;
    }
    bool valid = false;
    double dist = 0.0;
    if (i < scan_n(P)) {
        const int32_t* nb = P.kd_nbr + 5 * static_cast<size_t>(i);
        if (nb[0] == -3) atomicOr(&st->kd_tie, 1u);                 // k_knn_all: a deciding tie (the host reruns)
        if (nb[0] >= 0) {
            double Pm[5][3];
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const float4 v = P.kd_pts[nb[k]];
                Pm[k][0] = v.x; Pm[k][1] = v.y; Pm[k][2] = v.z;
            }
            // is_collinear(p0, p1, p2, 0.5) (:785-792): |normalize(p1-p0) x normalize(p2-p0)| < 0.5 rejects
            double v1[3], v2[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) { v1[d] = Pm[1][d] - Pm[0][d]; v2[d] = Pm[2][d] - Pm[0][d]; }
            const double n1 = sqrt(dot3d(v1[0], v1[1], v1[2], v1[0], v1[1], v1[2]));
            const double n2 = sqrt(dot3d(v2[0], v2[1], v2[2], v2[0], v2[1], v2[2]));
            if (n1 > 0) { v1[0] /= n1; v1[1] /= n1; v1[2] /= n1; }
            if (n2 > 0) { v2[0] /= n2; v2[1] /= n2; v2[2] /= n2; }
            const double cr0 = v1[1] * v2[2] - v1[2] * v2[1], cr1 = v1[2] * v2[0] - v1[0] * v2[2],
                         cr2 = v1[0] * v2[1] - v1[1] * v2[0];
            if (!(sqrt(dot3d(cr0, cr1, cr2, cr0, cr1, cr2)) < 0.5)) {
                double cen[3] = {0.0, 0.0, 0.0};
#pragma unroll
                for (int k = 0; k < 5; ++k) { cen[0] += Pm[k][0]; cen[1] += Pm[k][1]; cen[2] += Pm[k][2]; }
                cen[0] /= 5.0; cen[1] /= 5.0; cen[2] /= 5.0;
                double S[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
                for (int k = 0; k < 5; ++k) {
                    const double a[3] = {Pm[k][0] - cen[0], Pm[k][1] - cen[1], Pm[k][2] - cen[2]};
#pragma unroll
                    for (int r = 0; r < 3; ++r)
#pragma unroll
                        for (int s = 0; s < 3; ++s) S[r][s] += a[r] * a[s];
                }
                double nrm[3];
                smallest_eigvec3d(S, nrm);
                float T[12];
#pragma unroll
                for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
                float qx, qy, qz;
                transform_pt(T, P.pts[3 * i], P.pts[3 * i + 1], P.pts[3 * i + 2], qx, qy, qz);
                const double pd = -dot3d(nrm[0], nrm[1], nrm[2], cen[0], cen[1], cen[2]);
                dist = fabs(dot3d(nrm[0], nrm[1], nrm[2], qx, qy, qz) + pd);
                valid = P.loop || !(dist > P.maxd);             // :746-748 (NaN kept); the loop ICP has no gate (:573)
                if (valid) {
                    Slot sl;
                    sl.key = 0;
#pragma unroll
                    for (int d = 0; d < 3; ++d) { sl.n[d] = static_cast<float>(nrm[d]); sl.c[d] = static_cast<float>(cen[d]); }
                    if (P.loop) {
                        // find_correspondences_loop keeps neighbour 0 in the matched keyframe's frame (T_lw in fp64,
                        // :517-520); optimize_loop casts it to fp32 and puts it back in the world, R_m p + t_m (:148-150)
                        float lf[3];
#pragma unroll
                        for (int r = 0; r < 3; ++r) {
                            const double l = ((static_cast<double>(P.Tlw[4 * r]) * Pm[0][0] +
                                               static_cast<double>(P.Tlw[4 * r + 1]) * Pm[0][1]) +
                                              static_cast<double>(P.Tlw[4 * r + 2]) * Pm[0][2]) + static_cast<double>(P.Tlw[4 * r + 3]);
                            lf[r] = static_cast<float>(l);
                        }
#pragma unroll
                        for (int r = 0; r < 3; ++r)
                            sl.c[r] = dot3f(P.Tm[4 * r], P.Tm[4 * r + 1], P.Tm[4 * r + 2], lf[0], lf[1], lf[2]) + P.Tm[4 * r + 3];
                    }
                    P.kd_plane[i] = sl;
                    P.kd_res[i] = dist;
                }
            }
        }
        P.slot[i] = valid ? i : -1;
        if (P.res_dbg) P.res_dbg[i] = valid ? dist : 0.0;
    }
    corr_epilogue(P, valid, dist, with_stats, blockIdx.x);
    if (P.presort)                                      // iteration 0, reference-exact mode (uniform branch)
        presort_block(P.presort, blockIdx.x, valid ? static_cast<uint64_t>(__double_as_longlong(dist)) : kInfKey);
}

// optimize_loop's inlier ratio (:206-238): the curr cloud at the converged pose (t + R p, :220-221), each point an
// inlier when its nearest matched-map point is closer than 1 m: sqrt of nanoflann's fp32 (dx^2 + dy^2) + dz^2 < 1.
// Every map point within 1 m lies in the cells spanned by q +- (1 m + kKnnMargin) (the margin covers the fp32
// rounding of q / h and of the grid's own cell index), so the grid answers the 1-NN threshold test exactly.  One
// lane per point, a row's points 8 loads at a time, early exit on a hit.
__global__ __launch_bounds__(kBlock) void k_inlier(KParams P) {
    DevState* st = P.st;
    const int i = blockIdx.x * kBlock + threadIdx.x;
    bool in = false;
    if (i < scan_n(P)) {
        float T[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
        const float px = P.pts[3 * i], py = P.pts[3 * i + 1], pz = P.pts[3 * i + 2];
        const float q[3] = {T[3] + dot3f(T[0], T[1], T[2], px, py, pz), T[7] + dot3f(T[4], T[5], T[6], px, py, pz),
                            T[11] + dot3f(T[8], T[9], T[10], px, py, pz)};
        if (isfinite(q[0]) && isfinite(q[1]) && isfinite(q[2]) && P.kd_m > 0) {
            int lo[3], hi[3];
            bool any = true;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const float rr = 1.0f + static_cast<float>(kKnnMargin);
                const float fl = floorf((q[a] - rr) / P.kd_h), fh = floorf((q[a] + rr) / P.kd_h);
                const float o = static_cast<float>(P.kd_org[a]), d = static_cast<float>(P.kd_dim[a]);
                const float l = fmaxf(fl - o, 0.0f), h = fminf(fh - o, d - 1.0f);
                if (!(l <= h)) any = false;
                lo[a] = any ? static_cast<int>(l) : 0;
                hi[a] = any ? static_cast<int>(h) : -1;
            }
            for (int z = lo[2]; any && !in && z <= hi[2]; ++z)
                for (int y = lo[1]; !in && y <= hi[1]; ++y) {
                    const size_t row = (static_cast<size_t>(z) * P.kd_dim[1] + y) * P.kd_dim[0];
                    const uint32_t b = P.kd_start[row + lo[0]], e = P.kd_start[row + hi[0] + 1];
                    for (uint32_t p0 = b; !in && p0 < e; p0 += 8) {
                        float4 v[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) v[u] = (p0 + u < e) ? P.kd_pts[p0 + u] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
                        for (int u = 0; u < 8; ++u) {
                            const float d0 = q[0] - v[u].x, d1 = q[1] - v[u].y, d2 = q[2] - v[u].z;
                            const float d = (d0 * d0 + d1 * d1) + d2 * d2;
                            in = in || (p0 + u < e && sqrtf(d) < 1.0f);
                        }
                    }
                }
        }
    }
    const uint64_t m = __ballot(in);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&st->inliers, static_cast<unsigned>(__popcll(m)));
}

}  // namespace lo
