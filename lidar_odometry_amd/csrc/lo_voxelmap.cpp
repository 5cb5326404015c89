// lo_voxelmap.cpp — host C++ map side (include/lo_map.h).
//
// The ICP kernels only read the surfel table; this file builds it the way the reference does so the
// product runs a full odometry loop without the reference: map::VoxelMap::UpdateVoxelMap
// (src/database/VoxelMap.cpp:128-262) and map::FastVoxelFilter::filter (src/database/VoxelMap.h:73-104).
//
// Result-defining details kept from the reference:
//  * containers iterate in insertion order and erase by moving the last element into the hole
//    (ankerl::unordered_dense do_erase) — this fixes the child order used in the fp32 centroid/covariance
//    sums and the order of L0 pruning;
//  * keys: PointToVoxelKey = floor(p / scale) with scale = voxel * factor in fp32 (:50-58); the L0->L1
//    parent is integer floor division (:60-67);
//  * the surfel normal is U.col(2) of Eigen's 2-sided Jacobi SVD of the fp32 covariance (restated below),
//    planarity = s2 / (s0 + 1e-6f) (:239-243).
#include <algorithm>
#include <atomic>
#include <mutex>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/lo_map.h"
#include "lo_ctx_internal.h"
#include "lo_math.h"

namespace lo {
namespace {

struct Key3 {
    int32_t x, y, z;
};
inline bool operator==(const Key3& a, const Key3& b) { return a.x == b.x && a.y == b.y && a.z == b.z; }

inline uint64_t mix64(uint64_t h) {
    __uint128_t r = static_cast<__uint128_t>(h) * 0x9E3779B97F4A7C15ull;
    return static_cast<uint64_t>(r) ^ static_cast<uint64_t>(r >> 64);
}
struct HashKey3 {
    uint64_t operator()(const Key3& k) const {
        const uint64_t xy = static_cast<uint64_t>(static_cast<uint32_t>(k.x)) << 32 | static_cast<uint32_t>(k.y);
        return mix64(xy ^ static_cast<uint64_t>(static_cast<uint32_t>(k.z)) * 0xD6E8FEB86659FD93ull);
    }
};
struct HashU64 {
    uint64_t operator()(uint64_t k) const { return mix64(k); }
};
struct NoValue {};

// Insertion-ordered open-addressing map; erase moves the last entry into the hole (the value order of
// ankerl::unordered_dense, which the reference iterates).  The index is linear probing at load <= 1/2 with the
// 32-bit hash cached in each slot, so a probe touches a key only on a hash match.
template <class K, class V, class H>
class OrderedMap {
  public:
    OrderedMap() { reindex(16); }
    size_t size() const { return keys_.size(); }
    bool empty() const { return keys_.empty(); }
    const K& key_at(size_t i) const { return keys_[i]; }
    V& val_at(size_t i) { return vals_[i]; }
    const V& val_at(size_t i) const { return vals_[i]; }

    int64_t find(const K& k) const {
        const uint32_t h = hash32(k);
        for (uint64_t b = h & mask_;; b = (b + 1) & mask_) {
            const Slot& e = slots_[b];
            if (e.idx < 0) return -1;
            if (e.h == h && keys_[e.idx] == k) return e.idx;
        }
    }
    // returns index; *inserted set when new (value default-constructed)
    size_t upsert(const K& k, bool* inserted) {
        const uint32_t h = hash32(k);
        uint64_t b = h & mask_;
        for (;; b = (b + 1) & mask_) {
            const Slot& e = slots_[b];
            if (e.idx < 0) break;
            if (e.h == h && keys_[e.idx] == k) { if (inserted) *inserted = false; return static_cast<size_t>(e.idx); }
        }
        keys_.push_back(k);
        vals_.emplace_back();
        const int32_t i = static_cast<int32_t>(keys_.size() - 1);
        if (keys_.size() * 2 > slots_.size()) reindex(slots_.size() * 2);
        else slots_[b] = {i, h};
        if (inserted) *inserted = true;
        return keys_.size() - 1;
    }
    bool erase(const K& k) {
        const uint32_t hk = hash32(k);
        uint64_t b = hk & mask_;
        for (;; b = (b + 1) & mask_) {
            const Slot& e = slots_[b];
            if (e.idx < 0) return false;
            if (e.h == hk && keys_[e.idx] == k) break;
        }
        const int32_t victim = slots_[b].idx;
        slots_[b].idx = -1;
        for (uint64_t j = (b + 1) & mask_; slots_[j].idx >= 0; j = (j + 1) & mask_) {   // backward shift
            const uint64_t home = slots_[j].h & mask_;
            if (((j - home) & mask_) >= ((j - b) & mask_)) { slots_[b] = slots_[j]; slots_[j].idx = -1; b = j; }
        }
        const int32_t last = static_cast<int32_t>(keys_.size() - 1);
        if (victim != last) {
            const uint32_t hl = hash32(keys_[last]);
            uint64_t s = hl & mask_;
            while (slots_[s].idx != last) s = (s + 1) & mask_;
            keys_[victim] = keys_[last];
            vals_[victim] = std::move(vals_[last]);
            slots_[s].idx = victim;
        }
        keys_.pop_back();
        vals_.pop_back();
        return true;
    }
    // empties the map but keeps the slot array (a per-update scratch map never re-grows from 16 slots)
    void clear() {
        keys_.clear();
        vals_.clear();
        std::fill(slots_.begin(), slots_.end(), Slot{-1, 0});
    }

  private:
    struct Slot {
        int32_t idx;
        uint32_t h;
    };
    static uint32_t hash32(const K& k) { return static_cast<uint32_t>(H()(k)); }
    void reindex(size_t cap) {
        slots_.assign(cap, Slot{-1, 0});
        mask_ = cap - 1;
        for (size_t i = 0; i < keys_.size(); ++i) {
            const uint32_t h = hash32(keys_[i]);
            uint64_t b = h & mask_;
            while (slots_[b].idx >= 0) b = (b + 1) & mask_;
            slots_[b] = {static_cast<int32_t>(i), h};
        }
    }
    std::vector<K> keys_;
    std::vector<V> vals_;
    std::vector<Slot> slots_;
    uint64_t mask_ = 0;
};

struct L0 {
    float c[3] = {0.0f, 0.0f, 0.0f};
    int hit_count = 1;
    int point_count = 0;
};

// occupied_children (ankerl::unordered_dense::set, VoxelMap.h:312-318): insertion order, erase moves the last
// element into the hole.  An L1 voxel has at most factor^3 children (27 at kitti.yaml's factor 3), so a linear
// list with the same order semantics replaces the hashed set (no per-voxel allocation, no rehash).
class ChildSet {
  public:
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    const Key3& key_at(size_t i) const { return data()[i]; }
    void upsert(const Key3& k, bool* fresh) {
        Key3* d = data();
        for (size_t i = 0; i < n_; ++i) if (d[i] == k) { if (fresh) *fresh = false; return; }
        if (n_ == kInline) { spill_.assign(inline_, inline_ + kInline); }
        if (n_ >= kInline) spill_.push_back(k); else inline_[n_] = k;
        ++n_;
        if (fresh) *fresh = true;
    }
    void erase(const Key3& k) {
        Key3* d = data();
        for (size_t i = 0; i < n_; ++i) {
            if (!(d[i] == k)) continue;
            d[i] = d[n_ - 1];
            --n_;
            if (n_ >= kInline) spill_.pop_back();
            else if (n_ == kInline - 1 && !spill_.empty()) { std::copy(spill_.begin(), spill_.begin() + n_, inline_); spill_.clear(); }
            return;
        }
    }

  private:
    static constexpr size_t kInline = 27;
    Key3* data() { return n_ > kInline || (n_ == kInline && !spill_.empty()) ? spill_.data() : inline_; }
    const Key3* data() const { return n_ > kInline || (n_ == kInline && !spill_.empty()) ? spill_.data() : inline_; }
    Key3 inline_[kInline];
    std::vector<Key3> spill_;
    size_t n_ = 0;
};
struct L1 {
    ChildSet children;
    bool has_surfel = false;
    float normal[3] = {0.0f, 0.0f, 0.0f};
    float centroid[3] = {0.0f, 0.0f, 0.0f};
    float planarity = 1.0f;
    int last_child_count = 0;
};

}  // namespace

struct HostVoxelMap {
    float voxel = 0.5f;
    int factor = 3;
    float planarity_thr = 0.1f;
    bool compute_surfels = true;
    OrderedMap<Key3, L0, HashKey3> l0;
    OrderedMap<Key3, L1, HashKey3> l1;

    OrderedMap<Key3, NoValue, HashKey3> touched;   // scratch, kept across updates
    std::vector<int32_t> k0, k1;
    // L1 keys whose surfel may have changed (created, refitted, lost, erased), in update order: a device table
    // synced at journal position p catches up by patching the keys of journal[p:] (lo_map_sync_voxelmap).  epoch
    // changes when the journal restarts, which forces a full upload.
    std::vector<Key3> journal;
    uint64_t epoch = 1;
    size_t changed_from = 0;                       // journal[changed_from:]: the keys the last update noted
    void note(const Key3& k) { journal.push_back(k); }

    // PointToVoxelKey for a whole cloud: floor(p / scale) per coordinate, one flat loop over the 3n floats
    // (vectorised: divps + roundps; the same IEEE division and floor as the per-point form)
    static void keys_of(const float* xyz, size_t n, float s, std::vector<int32_t>& out) {
        out.resize(3 * n);
        int32_t* o = out.data();
        for (size_t j = 0; j < 3 * n; ++j) o[j] = static_cast<int32_t>(std::floor(xyz[j] / s));
    }
    Key3 parent(const Key3& k) const {
        const int f = factor;
        auto d = [f](int v) { return v >= 0 ? v / f : (v - (f - 1)) / f; };
        return {d(k.x), d(k.y), d(k.z)};
    }
    void unregister(const Key3& k) {
        const Key3 p = parent(k);
        const int64_t i = l1.find(p);
        if (i < 0) return;
        note(p);
        L1& n = l1.val_at(i);
        n.children.erase(k);
        if (n.children.size() < 5) n.has_surfel = false;
        if (n.children.empty()) l1.erase(p);
    }
    void add_point(const float* p, const Key3& k) {
        bool fresh = false;
        const size_t i = l0.upsert(k, &fresh);
        L0& v = l0.val_at(i);
        const int n = v.point_count;
        if (n == 0) {
            std::memcpy(v.c, p, sizeof(float) * 3);
            v.hit_count = 1;
            v.point_count = 1;
        } else {
            const float nf = static_cast<float>(n), n1 = static_cast<float>(n + 1);
            for (int a = 0; a < 3; ++a) v.c[a] = (v.c[a] * nf + p[a]) / n1;
            v.point_count++;
        }
        if (fresh) {
            const size_t j = l1.upsert(parent(k), nullptr);
            l1.val_at(j).children.upsert(k, nullptr);
        }
    }

    // The L1 voxel's children's L0 centroids in child order
    void child_centroids(const L1& node, std::vector<float>& cs) const {
        cs.clear();
        for (size_t q = 0; q < node.children.size(); ++q) {
            const int64_t c0 = l0.find(node.children.key_at(q));
            if (c0 >= 0) cs.insert(cs.end(), l0.val_at(c0).c, l0.val_at(c0).c + 3);
        }
    }
    // Surfel fit (VoxelMap.cpp:211-243): fp32 mean and covariance in child order, JacobiSVD<Matrix3f> (restated),
    // normal = U.col(2); returns planarity = s2 / (s0 + 1e-6)
    static float fit(const std::vector<float>& cs, float cen[3], float U[3][3]) {
        return surfel_fit(cs.data(), static_cast<int>(cs.size() / 3), cen, U);
    }

    // Deferred fits (lo_voxelmap_set_device_fit): the touched loop of update() records each refit as a job (L1 key,
    // child count, child centroids in child order) instead of fitting; lo_map_sync_voxelmap runs the jobs on the
    // device (k_surfel_fit, which also patches the synced table), and resolve() applies the results in job order --
    // surfel fields, or on a planarity failure the erase of the voxel and its children, exactly where the sequential
    // loop would have done it (no other structural change happens in that loop, and the jobs' inputs are per voxel).
    // Every reader of the map resolves first; without a device result the jobs are fitted here.
    bool defer_fit = false;
    std::vector<Key3> job_key;
    std::vector<int32_t> job_cnt, job_off;               // child count; offset into job_cs (floats / 3)
    std::vector<float> job_cs;
    lo_ctx* fit_ctx = nullptr;                           // the context whose k_surfel_fit holds the results
    uint64_t fit_id = 0;                                 // its ticket
    void resolve() {
        if (job_key.empty()) return;
        const size_t nj = job_key.size();
        std::vector<FitResult> res(nj);
        bool have = fit_ctx && ctx_fit_results(fit_ctx, fit_id, res.data(), nj) == LO_OK;
        if (!have) {
            for (size_t j = 0; j < nj; ++j) {
                const int m = (j + 1 < nj ? job_off[j + 1] : static_cast<int32_t>(job_cs.size() / 3)) - job_off[j];
                float U[3][3];
                res[j].planarity = surfel_fit(job_cs.data() + 3 * job_off[j], m, res[j].c, U);
                for (int a = 0; a < 3; ++a) res[j].n[a] = U[a][2];
            }
        }
        for (size_t j = 0; j < nj; ++j) {
            const int64_t li = l1.find(job_key[j]);
            if (li < 0) continue;                           // cannot happen: jobs are unique, nothing erased them
            L1& node = l1.val_at(li);
            if (res[j].planarity > planarity_thr) {
                node.has_surfel = false;
                std::vector<Key3> kids;
                for (size_t q = 0; q < node.children.size(); ++q) kids.push_back(node.children.key_at(q));
                for (const Key3& k : kids) l0.erase(k);
                l1.erase(job_key[j]);
                continue;
            }
            node.has_surfel = true;
            for (int a = 0; a < 3; ++a) { node.normal[a] = res[j].n[a]; node.centroid[a] = res[j].c[a]; }
            node.planarity = res[j].planarity;
            node.last_child_count = job_cnt[j];
        }
        job_key.clear();
        job_cnt.clear();
        job_off.clear();
        job_cs.clear();
        fit_ctx = nullptr;
    }

    // VoxelMap::ApplyTransformAndRehash (VoxelMap.cpp:264-302), after a pose-graph correction: every L0 centroid
    // moved by T (R c + t, Matrix3f * Vector3f order) and re-keyed in L0 order, colliding voxels merged by point
    // count, the L1 level rebuilt from the new keys (RegisterToParent), then RecomputeAllSurfels (:304-366: at least
    // 5 children, planarity failures lose the surfel without being erased).  The device tables need a full upload
    // afterwards (the journal restarts).
    void apply_transform(const float T[12]) {
        resolve();
        const SE3f s = se3_from12(T);
        std::vector<std::pair<Key3, L0>> tr;
        tr.reserve(l0.size());
        for (size_t i = 0; i < l0.size(); ++i) {
            L0 nn = l0.val_at(i);
            const float* c = l0.val_at(i).c;
            for (int r = 0; r < 3; ++r) nn.c[r] = dot3e(s.R[r][0], s.R[r][1], s.R[r][2], c[0], c[1], c[2]) + s.t[r];
            const Key3 k{static_cast<int32_t>(std::floor(nn.c[0] / voxel)), static_cast<int32_t>(std::floor(nn.c[1] / voxel)),
                         static_cast<int32_t>(std::floor(nn.c[2] / voxel))};
            tr.emplace_back(k, nn);
        }
        l0.clear();
        l1.clear();
        for (const auto& kn : tr) {
            bool fresh = false;
            const size_t i = l0.upsert(kn.first, &fresh);
            L0& ex = l0.val_at(i);
            if (ex.point_count == 0) {
                ex = kn.second;
            } else {
                const float n1 = static_cast<float>(ex.point_count), n2 = static_cast<float>(kn.second.point_count);
                for (int a = 0; a < 3; ++a) ex.c[a] = (ex.c[a] * n1 + kn.second.c[a] * n2) / (n1 + n2);
                ex.point_count += kn.second.point_count;
            }
            const size_t j = l1.upsert(parent(kn.first), nullptr);
            l1.val_at(j).children.upsert(kn.first, nullptr);
        }
        journal.clear();
        ++epoch;
        changed_from = 0;                            // every key moved: a keyed sync cannot follow, upload it all
        if (!compute_surfels) return;
        std::vector<float> cs;
        for (size_t t = 0; t < l1.size(); ++t) {
            L1& node = l1.val_at(t);
            const int cnt = static_cast<int>(node.children.size());
            if (cnt < 5) { node.has_surfel = false; continue; }
            child_centroids(node, cs);
            if (cs.size() / 3 < 5) { node.has_surfel = false; continue; }
            float U[3][3], cen[3];
            const float planarity = fit(cs, cen, U);
            if (planarity > planarity_thr) { node.has_surfel = false; continue; }
            node.has_surfel = true;
            for (int a = 0; a < 3; ++a) { node.normal[a] = U[a][2]; node.centroid[a] = cen[a]; }
            node.planarity = planarity;
            node.last_child_count = cnt;
        }
    }

    void update(const float* xyz, size_t n, const double sensor[3], double max_distance, bool keyframe) {
        resolve();
        changed_from = journal.size();               // nothing changed unless this update changes it
        if (!xyz || n == 0 || !keyframe) return;
        if (journal.size() > (size_t(1) << 22)) { journal.clear(); ++epoch; changed_from = 0; }
        const float sp[3] = {static_cast<float>(sensor[0]), static_cast<float>(sensor[1]), static_cast<float>(sensor[2])};
        const float rsq = static_cast<float>(max_distance * max_distance);
        std::vector<Key3> doomed;
        for (size_t i = 0; i < l0.size(); ++i) {
            const float* c = l0.val_at(i).c;
            const float d0 = c[0] - sp[0], d1 = c[1] - sp[1], d2 = c[2] - sp[2];
            const float e0 = d0 * d0, e1 = d1 * d1, e2 = d2 * d2;
            if (e0 + (e1 + e2) > rsq) doomed.push_back(l0.key_at(i));
        }
        for (const Key3& k : doomed) { unregister(k); l0.erase(k); }
        std::vector<Key3> empty1;
        for (size_t i = 0; i < l1.size(); ++i) if (l1.val_at(i).children.empty()) empty1.push_back(l1.key_at(i));
        for (const Key3& k : empty1) { note(k); l1.erase(k); }

        keys_of(xyz, n, voxel, k0);
        keys_of(xyz, n, voxel * static_cast<float>(factor), k1);
        touched.clear();
        for (size_t i = 0; i < n; ++i) {
            add_point(xyz + 3 * i, Key3{k0[3 * i], k0[3 * i + 1], k0[3 * i + 2]});
            touched.upsert(Key3{k1[3 * i], k1[3 * i + 1], k1[3 * i + 2]}, nullptr);
        }
        if (!compute_surfels) return;
        std::vector<float> cs;
        for (size_t t = 0; t < touched.size(); ++t) {
            const Key3 k1 = touched.key_at(t);
            const int64_t li = l1.find(k1);
            if (li < 0) continue;
            L1& node = l1.val_at(li);
            const int cnt = static_cast<int>(node.children.size());
            if (cnt < 5) {
                if (node.has_surfel) note(k1);                 // loses its surfel
                node.has_surfel = false;
                continue;
            }
            if (node.has_surfel && node.last_child_count == cnt) continue;
            note(k1);                                          // refitted, erased or losing its surfel below
            child_centroids(node, cs);
            if (cs.size() / 3 < 3) { node.has_surfel = false; continue; }
            if (defer_fit) {                                   // resolve() finishes this voxel
                job_key.push_back(k1);
                job_cnt.push_back(cnt);
                job_off.push_back(static_cast<int32_t>(job_cs.size() / 3));
                job_cs.insert(job_cs.end(), cs.begin(), cs.end());
                node.has_surfel = false;
                continue;
            }
            float U[3][3], cen[3];
            const float planarity = fit(cs, cen, U);
            if (planarity > planarity_thr) {
                node.has_surfel = false;
                std::vector<Key3> kids;
                for (size_t q = 0; q < node.children.size(); ++q) kids.push_back(node.children.key_at(q));
                for (const Key3& k : kids) l0.erase(k);
                l1.erase(k1);
                continue;
            }
            node.has_surfel = true;
            for (int a = 0; a < 3; ++a) { node.normal[a] = U[a][2]; node.centroid[a] = cen[a]; }
            node.planarity = planarity;
            node.last_child_count = cnt;
        }
    }
};

}  // namespace lo

using lo::HostVoxelMap;

// Every entry point locks the map's recursive mutex, as the reference guards VoxelMap (VoxelMap.h: m_mutex): the
// const readers resolve pending device fits (erasing voxels, syncing an event), so they mutate too.  id is unique
// per map for the life of the process (a context's incremental sync names its source by it: an address can be
// recycled by the next map).
static std::atomic<uint64_t> g_map_ids{1};
struct lo_voxelmap {
    HostVoxelMap m;
    std::recursive_mutex mu;
    const uint64_t id = g_map_ids.fetch_add(1);
};
#define LO_MAP_LOCK(m) std::lock_guard<std::recursive_mutex> lo_map_guard_(const_cast<lo_voxelmap*>(m)->mu)

// Readers see the map as the sequential UpdateVoxelMap leaves it: pending device fits are applied first.
static const HostVoxelMap& resolved(const lo_voxelmap* m) {
    HostVoxelMap& h = const_cast<lo_voxelmap*>(m)->m;
    h.resolve();
    return h;
}

extern "C" {

lo_voxelmap* lo_voxelmap_create(float voxel_size, int hierarchy_factor, float planarity_threshold, int compute_surfels) {
    if (!(voxel_size > 0.0f) || hierarchy_factor <= 0 || hierarchy_factor % 2 == 0) return nullptr;
    lo_voxelmap* v = new lo_voxelmap();
    v->m.voxel = voxel_size;
    v->m.factor = hierarchy_factor;
    v->m.planarity_thr = planarity_threshold;
    v->m.compute_surfels = compute_surfels != 0;
    return v;
}

void lo_voxelmap_destroy(lo_voxelmap* m) { delete m; }

int lo_voxelmap_apply_transform(lo_voxelmap* m, const float T[12]) {
    if (!m || !T) return LO_ERR_ARG;
    LO_MAP_LOCK(m);
    m->m.apply_transform(T);
    return LO_OK;
}

int lo_voxelmap_update(lo_voxelmap* m, const float* xyz, size_t n, const double sensor[3], double max_distance, int is_keyframe) {
    if (!m || !sensor || (n > 0 && !xyz)) return LO_ERR_ARG;
    LO_MAP_LOCK(m);
    m->m.update(xyz, n, sensor, max_distance, is_keyframe != 0);
    return LO_OK;
}

size_t lo_voxelmap_l0_count(const lo_voxelmap* m) {
    if (!m) return 0;
    LO_MAP_LOCK(m);
    return resolved(m).l0.size();
}
size_t lo_voxelmap_l1_count(const lo_voxelmap* m) {
    if (!m) return 0;
    LO_MAP_LOCK(m);
    return resolved(m).l1.size();
}
size_t lo_voxelmap_surfel_count(const lo_voxelmap* m) {
    if (!m) return 0;
    LO_MAP_LOCK(m);
    const HostVoxelMap& h = resolved(m);
    size_t c = 0;
    for (size_t i = 0; i < h.l1.size(); ++i) c += h.l1.val_at(i).has_surfel ? 1 : 0;
    return c;
}

int lo_voxelmap_set_device_fit(lo_voxelmap* m, int enable) {
    if (!m) return LO_ERR_ARG;
    LO_MAP_LOCK(m);
    m->m.resolve();
    m->m.defer_fit = enable != 0;
    return LO_OK;
}

size_t lo_voxelmap_get_surfels(const lo_voxelmap* m, int32_t* keys, float* normals, float* centroids, float* planarity, size_t cap) {
    if (!m) return 0;
    LO_MAP_LOCK(m);
    const HostVoxelMap& h = resolved(m);
    size_t c = 0;
    for (size_t i = 0; i < h.l1.size() && c < cap; ++i) {
        const auto& n = h.l1.val_at(i);
        if (!n.has_surfel) continue;
        const auto& k = h.l1.key_at(i);
        if (keys) { keys[3 * c] = k.x; keys[3 * c + 1] = k.y; keys[3 * c + 2] = k.z; }
        for (int a = 0; a < 3; ++a) {
            if (normals) normals[3 * c + a] = n.normal[a];
            if (centroids) centroids[3 * c + a] = n.centroid[a];
        }
        if (planarity) planarity[c] = n.planarity;
        ++c;
    }
    return c;
}

size_t lo_voxelmap_changed_l1(const lo_voxelmap* m, int32_t* keys, size_t cap) {
    if (!m) return 0;
    LO_MAP_LOCK(m);
    const HostVoxelMap& h = resolved(m);
    const size_t from = std::min(h.changed_from, h.journal.size());
    // each key once (a voxel can be noted by the prune and by the touched loop), ordered by its packed bits
    std::vector<uint64_t> u;
    u.reserve(h.journal.size() - from);
    for (size_t i = from; i < h.journal.size(); ++i) {
        const lo::Key3& k = h.journal[i];
        u.push_back((static_cast<uint64_t>(static_cast<uint32_t>(k.x)) << 42) ^
                    (static_cast<uint64_t>(static_cast<uint32_t>(k.y)) << 21) ^ static_cast<uint32_t>(k.z));
    }
    std::vector<size_t> idx(u.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return u[a] < u[b] || (u[a] == u[b] && a < b); });
    size_t cnt = 0;
    for (size_t r = 0; r < idx.size(); ++r) {
        if (r > 0 && u[idx[r]] == u[idx[r - 1]]) {
            const lo::Key3& a = h.journal[from + idx[r]];
            const lo::Key3& b = h.journal[from + idx[r - 1]];
            if (a == b) continue;                                  // (the packing is not injective: compare keys)
        }
        if (keys && cnt < cap) {
            const lo::Key3& k = h.journal[from + idx[r]];
            keys[3 * cnt] = k.x; keys[3 * cnt + 1] = k.y; keys[3 * cnt + 2] = k.z;
        }
        ++cnt;
    }
    return cnt;
}

// GetSurfelAtPoint (VoxelMap.cpp:368-386): PointToVoxelKey(p, 1) (:50-58: fp32 scale voxel * factor, floor of the
// division), then the L1 voxel's surfel if it has one
int lo_voxelmap_surfel_at(const lo_voxelmap* m, const float p[3], float normal[3], float centroid[3]) {
    if (!m || !p) return 0;
    LO_MAP_LOCK(m);
    const HostVoxelMap& h = resolved(m);
    const float scale = h.voxel * static_cast<float>(h.factor);
    const lo::Key3 k{static_cast<int>(std::floor(p[0] / scale)), static_cast<int>(std::floor(p[1] / scale)),
                 static_cast<int>(std::floor(p[2] / scale))};
    const int64_t i = h.l1.find(k);
    if (i < 0 || !h.l1.val_at(i).has_surfel) return 0;
    const lo::L1& node = h.l1.val_at(i);
    for (int a = 0; a < 3; ++a) {
        if (normal) normal[a] = node.normal[a];
        if (centroid) centroid[a] = node.centroid[a];
    }
    return 1;
}

size_t lo_voxelmap_surfels_at_keys(const lo_voxelmap* m, const int32_t* keys, size_t n, float* normals, float* centroids,
                                   uint8_t* present) {
    if (!m || (n > 0 && (!keys || !normals || !centroids || !present))) return 0;
    LO_MAP_LOCK(m);
    const HostVoxelMap& h = resolved(m);
    const float l1 = h.voxel * static_cast<float>(h.factor);
    size_t found = 0;
    for (size_t i = 0; i < n; ++i) {
        // GetSurfelAtPoint at the key's voxel centre: PointToVoxelKey(centre, 1) is the key itself
        const float c[3] = {(static_cast<float>(keys[3 * i]) + 0.5f) * l1, (static_cast<float>(keys[3 * i + 1]) + 0.5f) * l1,
                            (static_cast<float>(keys[3 * i + 2]) + 0.5f) * l1};
        const lo::Key3 k{static_cast<int>(std::floor(c[0] / l1)), static_cast<int>(std::floor(c[1] / l1)),
                         static_cast<int>(std::floor(c[2] / l1))};
        const int64_t j = h.l1.find(k);
        const bool has = j >= 0 && h.l1.val_at(j).has_surfel;
        present[i] = has ? 1 : 0;
        for (int a = 0; a < 3; ++a) {
            normals[3 * i + a] = has ? h.l1.val_at(j).normal[a] : 0.0f;
            centroids[3 * i + a] = has ? h.l1.val_at(j).centroid[a] : 0.0f;
        }
        found += has ? 1 : 0;
    }
    return found;
}

size_t lo_voxelmap_get_l0(const lo_voxelmap* m, float* xyz, size_t cap) {
    if (!m || !xyz) return 0;
    LO_MAP_LOCK(m);
    const HostVoxelMap& h = resolved(m);
    size_t c = 0;
    for (; c < h.l0.size() && c < cap; ++c) std::memcpy(xyz + 3 * c, h.l0.val_at(c).c, sizeof(float) * 3);
    return c;
}

int lo_map_sync_voxelmap(lo_ctx* ctx, const lo_voxelmap* m, int* patched) {
    if (!ctx || !m) return LO_ERR_ARG;
    if (patched) *patched = -1;
    lo_config cfg;
    if (lo_get_config(ctx, &cfg) != LO_OK) return LO_ERR_ARG;
    LO_MAP_LOCK(m);
    HostVoxelMap& H = const_cast<lo_voxelmap*>(m)->m;
    if (cfg.use_surfel_correspondence) {
        uint64_t src = 0, epoch = 0, pos = 0;
        lo::ctx_map_source(ctx, &src, &epoch, &pos);
        if (H.fit_ctx) H.resolve();                     // fits already handed to a context: collect them first
        if (src == m->id && epoch == H.epoch && pos <= H.journal.size()) {
            // the changed L1 keys, once each; keys with a pending fit job are patched by k_surfel_fit after these
            lo::OrderedMap<lo::Key3, lo::NoValue, lo::HashKey3> jobs;
            for (const lo::Key3& k : H.job_key) jobs.upsert(k, nullptr);
            lo::OrderedMap<lo::Key3, lo::NoValue, lo::HashKey3> keys;
            for (size_t i = pos; i < H.journal.size(); ++i)
                if (jobs.find(H.journal[i]) < 0) keys.upsert(H.journal[i], nullptr);
            const size_t cnt = keys.size();
            std::vector<int32_t> k(3 * std::max<size_t>(cnt, 1));
            std::vector<float> nn(3 * std::max<size_t>(cnt, 1)), cc(3 * std::max<size_t>(cnt, 1));
            std::vector<uint8_t> present(std::max<size_t>(cnt, 1));
            for (size_t i = 0; i < cnt; ++i) {
                const lo::Key3& kk = keys.key_at(i);
                k[3 * i] = kk.x; k[3 * i + 1] = kk.y; k[3 * i + 2] = kk.z;
                const int64_t li = H.l1.find(kk);
                const bool has = li >= 0 && H.l1.val_at(li).has_surfel;
                present[i] = has ? 1 : 0;
                for (int a = 0; a < 3; ++a) {
                    nn[3 * i + a] = has ? H.l1.val_at(li).normal[a] : 0.0f;
                    cc[3 * i + a] = has ? H.l1.val_at(li).centroid[a] : 0.0f;
                }
            }
            int rc = lo_map_patch_surfels(ctx, k.data(), nn.data(), cc.data(), present.data(), cnt);
            if (rc == LO_OK && !H.job_key.empty()) {
                const size_t nj = H.job_key.size();
                std::vector<int32_t> jk(3 * nj);
                for (size_t j = 0; j < nj; ++j) { jk[3 * j] = H.job_key[j].x; jk[3 * j + 1] = H.job_key[j].y; jk[3 * j + 2] = H.job_key[j].z; }
                uint64_t id = 0;
                rc = lo::ctx_fit_surfels(ctx, jk.data(), H.job_off.data(), nj, H.job_cs.data(), H.job_cs.size() / 3,
                                         H.planarity_thr, &id);
                if (rc == LO_OK) { H.fit_ctx = ctx; H.fit_id = id; }
            }
            if (rc == LO_OK) {
                lo::ctx_set_map_source(ctx, m->id, H.epoch, H.journal.size());
                if (patched) *patched = static_cast<int>(cnt + H.job_key.size());
                return LO_OK;
            }
            if (rc != LO_ERR_CAPACITY) return rc;           // capacity: the table is rebuilt below
        }
    }
    H.resolve();                                         // a full upload needs the fitted surfels on the host
    const int rc = lo_map_set_from_voxelmap(ctx, m);
    if (rc == LO_OK && cfg.use_surfel_correspondence)
        lo::ctx_set_map_source(ctx, m->id, H.epoch, H.journal.size());
    return rc;
}

int lo_map_set_from_voxelmap(lo_ctx* ctx, const lo_voxelmap* m) {
    if (!ctx || !m) return LO_ERR_ARG;
    LO_MAP_LOCK(m);
    const size_t s = lo_voxelmap_surfel_count(m);
    std::vector<int32_t> k(3 * std::max<size_t>(s, 1));
    std::vector<float> n(3 * std::max<size_t>(s, 1)), c(3 * std::max<size_t>(s, 1));
    lo_voxelmap_get_surfels(m, k.data(), n.data(), c.data(), nullptr, s);
    int rc = lo_map_set_surfels(ctx, k.data(), n.data(), c.data(), s);
    if (rc != LO_OK) return rc;
    lo_config cfg;
    if (lo_get_config(ctx, &cfg) == LO_OK && !cfg.use_surfel_correspondence) {
        // KDTree variant: GetPointCloud (VoxelMap.cpp:388-403) in L0 order, then RebuildKdTree's grid
        const size_t l0 = lo_voxelmap_l0_count(m);
        std::vector<float> xyz(3 * std::max<size_t>(l0, 1));
        lo_voxelmap_get_l0(m, xyz.data(), l0);
        rc = lo_map_set_points(ctx, xyz.data(), l0);
    }
    return rc;
}

// FastVoxelFilter::filter (VoxelMap.h:73-104): Morton key of floor(p * (1/voxel)) + 2^20 clamped to 21 bits,
// running fp32 sums in input order, centroid = sum * (1/count); output in first-occurrence order.
size_t lo_voxel_filter(const float* in, size_t n, float voxel_size, int stride, float* out) {
    if (!in || !out || n == 0 || stride < 1) return 0;
    struct Acc { float sx = 0.0f, sy = 0.0f, sz = 0.0f; uint32_t count = 0; };
    lo::OrderedMap<uint64_t, Acc, lo::HashU64> acc;
    const float inv = 1.0f / voxel_size;
    auto expand = [](uint64_t v) {
        v &= 0x1FFFFF;
        v = (v | (v << 32)) & 0x1F00000000FFFFull;
        v = (v | (v << 16)) & 0x1F0000FF0000FFull;
        v = (v | (v << 8)) & 0x100F00F00F00F00Full;
        v = (v | (v << 4)) & 0x10C30C30C30C30C3ull;
        v = (v | (v << 2)) & 0x1249249249249249ull;
        return v;
    };
    for (size_t i = 0; i < n; i += static_cast<size_t>(stride)) {
        const float* p = in + 3 * i;
        if (!std::isfinite(p[0]) || !std::isfinite(p[1]) || !std::isfinite(p[2])) continue;
        int64_t q[3];
        for (int a = 0; a < 3; ++a) {
            q[a] = static_cast<int64_t>(std::floor(p[a] * inv)) + (1 << 20);
            q[a] = std::max<int64_t>(0, std::min<int64_t>(q[a], (1 << 21) - 1));
        }
        const uint64_t key = expand(static_cast<uint64_t>(q[0])) | (expand(static_cast<uint64_t>(q[1])) << 1) |
                             (expand(static_cast<uint64_t>(q[2])) << 2);
        Acc& a = acc.val_at(acc.upsert(key, nullptr));
        a.sx += p[0];
        a.sy += p[1];
        a.sz += p[2];
        a.count++;
    }
    for (size_t i = 0; i < acc.size(); ++i) {
        const Acc& a = acc.val_at(i);
        const float ic = 1.0f / static_cast<float>(a.count);
        out[3 * i] = a.sx * ic;
        out[3 * i + 1] = a.sy * ic;
        out[3 * i + 2] = a.sz * ic;
    }
    return acc.size();
}

}  // extern "C"
