// lo_kdorder.h — the visit order of the reference's kd-tree, for the KDTree variant's tie-breaks (host side).
//
// The reference's 5-NN is nanoflann 1.7.1 (util::KdTree, PointCloudUtils.h:370-423: KDTreeSingleIndexAdaptor,
// L2_Simple_Adaptor<float>, leaf size 10, built over VoxelMap::GetPointCloud at RebuildKdTree, VoxelMap.cpp:420-438).
// Its result is the five smallest by (fp32 squared distance, visit order): KNNResultSet::addPoint
// (nanoflann.hpp:234-267) keeps the earlier-visited point among equal distances, because NANOFLANN_FIRST_MATCH is
// not defined.  The device search (lo_kdtree.hip) is a grid search, not a tree walk, so equal distances are ranked
// with this tree's order: the same index construction as nanoflann's buildIndex -- divideTree / middleSplit_ /
// planeSplit (:1149-1210, :1320-1427) -- and, per point, its position in the reordered index array vAcc_.  For a
// query, searchLevel (:1885-1960) enters the child on the query's side of a node first ((q - divlow) +
// (q - divhigh) < 0 -> child1), and a leaf's points in vAcc_ order; kd_visit_before() in lo_kdtree.hip evaluates
// exactly that at the node that separates two tied points.
#pragma once
#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace lo {

struct KdNode {              // device layout (24 B); node 0 is the root
    int32_t child1;          // -1: leaf
    int32_t child2;
    uint32_t mid;            // vAcc_ positions [.., mid) under child1, [mid, ..) under child2
    int32_t divfeat;
    float divlow;            // child1's largest coordinate on divfeat
    float divhigh;           // child2's smallest coordinate on divfeat
};
static_assert(sizeof(KdNode) == 24, "KdNode layout");

class KdOrderBuilder {
public:
    // xyz: m points, AoS float3, in the cloud's index order (the index nanoflann reports)
    KdOrderBuilder(const float* xyz, size_t m) : p_(xyz), m_(m) {}

    void build(std::vector<KdNode>& nodes, std::vector<uint32_t>& vpos) {
        nodes.clear();
        vpos.assign(m_, 0);
        if (m_ == 0) return;
        acc_.resize(m_);
        for (size_t i = 0; i < m_; ++i) acc_[i] = static_cast<uint32_t>(i);
        for (int d = 0; d < 3; ++d) {                       // coordinates by vAcc_ position, permuted alongside it
            co_[d].resize(m_);
            for (size_t i = 0; i < m_; ++i) co_[d][i] = p_[3 * i + d];
        }
        Box bb;                                             // computeBoundingBox (:1845-1880)
        for (int d = 0; d < 3; ++d) bb.lo[d] = bb.hi[d] = at(0, d);
        for (size_t k = 1; k < m_; ++k)
            for (int d = 0; d < 3; ++d) {
                const float v = at(k, d);
                if (v < bb.lo[d]) bb.lo[d] = v;
                if (v > bb.hi[d]) bb.hi[d] = v;
            }
        nodes_ = &nodes;
        divide(0, m_, bb);
        for (size_t i = 0; i < m_; ++i) vpos[acc_[i]] = static_cast<uint32_t>(i);
    }

private:
    struct Box { float lo[3], hi[3]; };
    const float* p_;
    size_t m_;
    std::vector<uint32_t> acc_;
    std::vector<float> co_[3];                             // co_[d][k] = coordinate d of point acc_[k]
    std::vector<KdNode>* nodes_ = nullptr;

    float at(size_t k, int d) const { return co_[d][k]; }   // by position in acc_
    void swap_at(size_t a, size_t b) {
        std::swap(acc_[a], acc_[b]);
        for (int d = 0; d < 3; ++d) std::swap(co_[d][a], co_[d][b]);
    }

    int divide(size_t left, size_t right, Box& bb) {
        std::vector<KdNode>& N = *nodes_;
        const int id = static_cast<int>(N.size());
        N.push_back(KdNode{-1, -1, 0, 0, 0.0f, 0.0f});
        if (right - left <= 10) {                           // leaf: its points' extent
            for (int d = 0; d < 3; ++d) bb.lo[d] = bb.hi[d] = at(left, d);
            for (size_t k = left + 1; k < right; ++k)
                for (int d = 0; d < 3; ++d) {
                    const float v = at(k, d);
                    if (bb.lo[d] > v) bb.lo[d] = v;
                    if (bb.hi[d] < v) bb.hi[d] = v;
                }
            return id;
        }
        size_t idx;
        int f;
        float cut;
        middle_split(left, right - left, bb, idx, f, cut);
        Box lb = bb, rb = bb;
        lb.hi[f] = cut;
        const int c1 = divide(left, left + idx, lb);
        rb.lo[f] = cut;
        const int c2 = divide(left + idx, right, rb);
        KdNode& nd = N[id];
        nd.child1 = c1;
        nd.child2 = c2;
        nd.mid = static_cast<uint32_t>(left + idx);
        nd.divfeat = f;
        nd.divlow = lb.hi[f];
        nd.divhigh = rb.lo[f];
        for (int d = 0; d < 3; ++d) {
            bb.lo[d] = std::min(lb.lo[d], rb.lo[d]);
            bb.hi[d] = std::max(lb.hi[d], rb.hi[d]);
        }
        return id;
    }

    // among the axes whose (inherited) box span is within 1e-5 of the largest, the one whose points spread most;
    // cut at the box middle clamped to the points' range; balanced split index as nanoflann chooses it
    void middle_split(size_t ind, size_t count, const Box& bb, size_t& index, int& f, float& cut) {
        const float eps = static_cast<float>(0.00001);
        float max_span = bb.hi[0] - bb.lo[0];
        for (int d = 1; d < 3; ++d) max_span = std::max(max_span, bb.hi[d] - bb.lo[d]);
        float best_spread = -1.0f, mn_f = 0.0f, mx_f = 0.0f;
        f = 0;
        for (int d = 0; d < 3; ++d) {
            if (!(bb.hi[d] - bb.lo[d] >= (1 - eps) * max_span)) continue;
            const float* c = co_[d].data() + ind;
            float mn = c[0], mx = mn;
            for (size_t k = 1; k < count; ++k) {
                const float v = c[k];
                mn = v < mn ? v : mn;
                mx = v > mx ? v : mx;
            }
            if (mx - mn > best_spread) { f = d; best_spread = mx - mn; mn_f = mn; mx_f = mx; }
        }
        const float mid = (bb.lo[f] + bb.hi[f]) / 2;
        cut = mid < mn_f ? mn_f : (mid > mx_f ? mx_f : mid);
        size_t lim1, lim2;
        partition(ind, count, f, cut, lim1, lim2);
        index = lim1 > count / 2 ? lim1 : (lim2 < count / 2 ? lim2 : count / 2);
    }

    // planeSplit: [< cut | == cut | > cut] by two in-place swap passes (the swap pattern fixes vAcc_ order)
    void partition(size_t ind, size_t count, int f, float cut, size_t& lim1, size_t& lim2) {
        const float* c = co_[f].data() + ind;
        auto v = [&](size_t k) { return c[k]; };
        size_t l = 0, r = count - 1;
        for (;;) {
            while (l <= r && v(l) < cut) ++l;
            while (r && l <= r && v(r) >= cut) --r;
            if (l > r || !r) break;
            swap_at(ind + l, ind + r);
            ++l;
            --r;
        }
        lim1 = l;
        r = count - 1;
        for (;;) {
            while (l <= r && v(l) <= cut) ++l;
            while (r && l <= r && v(r) > cut) --r;
            if (l > r || !r) break;
            swap_at(ind + l, ind + r);
            ++l;
            --r;
        }
        lim2 = l;
    }
};

}  // namespace lo
