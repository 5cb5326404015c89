// lo_devmap.hip — the voxel map's keyframe update on the device (include/lo_map.h lo_devmap_*).
//
// map::VoxelMap::UpdateVoxelMap (src/database/VoxelMap.cpp:128-262) with AddPoint (:99-120), Register/Unregister
// (:69-97) and ApplyTransformAndRehash + RecomputeAllSurfels (:264-366), kept resident in HBM next to the ICP
// context whose surfel table it maintains.  The host map (lo_voxelmap.cpp, pinned to ankerl::unordered_dense's
// orders by tests/test_map_side.py) is the specification; this produces the same containers bit for bit:
//
//   * L0 / L1 are insertion-ordered arrays (the value vectors of unordered_dense) with a device hash index
//     key -> position each.  Erasing by key moves the LAST element into the hole (do_erase).  A batch of erases in
//     a given order is replayed by one lane on positions only (erase_sim: the tail region and the hole contents in
//     LDS), then applied in parallel (holes filled from the tail survivors, index entries moved / tombstoned);
//   * the radius prune (:146-169) marks in parallel, compacts the doomed positions in L0 order, unregisters them
//     from their parents (one lane per parent, its doomed children in L0 order: the children set's swap-erase), and
//     erases L0 in that order and the L1s that became empty in the order they emptied;
//   * AddPoint groups the points by L0 key in point order: new keys are appended in first-occurrence order, every
//     voxel's running mean (c n + p) / (n + 1) runs over its points in point order, new L0s register with their
//     parent in creation order (new L1s appended at their first child); the touched L1 set is the points' L1 keys in
//     first-occurrence order;
//   * each touched L1's refit only reads its own children's centroids, so all fits run in parallel (surfel_fit, the
//     host's own fp32 code); the planarity failures' erases (the voxel's children in child order, then the voxel)
//     are replayed in touched order;
//   * the ICP table (the context's Slot table, lookup_surfel) is patched for every L1 key the update changed.
// Host work per keyframe: ten kernel launches.  Surfel mode only; factor <= 3 (27 children per L1 voxel).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lo_map.h"
#include "lo_ctx_internal.h"
#include "lo_device.h"
#include "lo_math.h"

namespace lo {
namespace dm {

constexpr int kKids = 27;               // children per L1 voxel at factor 3
constexpr int kOrch = 1024;             // threads of the single-workgroup phases
constexpr int kPar = 256;               // threads of the parallel phases
constexpr int kPruneBlocks = 1024;      // workgroups of the prune mark / compaction
constexpr int kSimLds = 3840;           // erase batches up to this size replay in LDS (4 arrays per map level)
constexpr int kU = 4;                   // items per thread issued together in the single-workgroup phases
constexpr uint64_t kEmpty = ~0ull;
constexpr uint64_t kTomb = ~0ull - 1;

struct DmPose { float v[12]; };

enum Cnt {                              // device counters (DM::cnt)
    C_N0 = 0, C_N1, C_ERR, C_TOMB0, C_TOMB1, C_Q, C_NT, C_NCHG, C_TTOMB, C_REBUILD, C_NNEW, C_NL1, C_ABORT, C_COUNT
};
constexpr int kChunk = 256;             // workgroups of the chunked (ordered) point / new-voxel passes
enum Err { E_CAP0 = 1, E_CAP1 = 2, E_KIDS = 4, E_KEY = 8, E_LOST = 16 };
enum Rebuild { R_I0 = 1, R_I1 = 2, R_TAB = 4 };

struct DM {
    int C0, C1, NP;
    uint32_t h0l, h1l, hpl;              // log2 capacities: L0 index, L1 index, per-update point / parent hashes
    float voxel, l1scale, thr;
    int factor;
    int surfels;                         // SetComputeSurfels (Estimator.cpp:79): 0 for a KDTree-mode context -- no
                                         //   surfel decisions, so no planarity erases (VoxelMap.cpp:182-185)
    // L0 (insertion order)
    uint64_t* k0;
    float* c0;                           // xyz per voxel
    int* n0p;                            // point_count
    // L1 (insertion order)
    uint64_t* k1;
    uint64_t* kids;                      // kKids per voxel, child order
    int* nk;
    int* has;
    float* nrm;
    float* cen;
    float* plan;
    int* last;
    // indices key -> position
    uint64_t* i0k;
    int* i0v;
    uint64_t* i1k;
    int* i1v;
    int* cnt;
    // prune
    int* flag;
    int* blkcnt;
    int* bc;                             // per-chunk counts / offsets of the ordered passes (3 x kChunk each)
    int* bo;
    int* D;                              // doomed L0 positions, L0 order
    int* emptied;                        // per doomed entry: the L1 position it emptied, or -1
    int* ucnt;                           // per L1 position: doomed children (zero between updates)
    int* ulist;                          // per L1 position: kKids doomed entries
    int* E1;                             // L1 erase list
    int* hole0;                          // erase replay outputs (indexed by position)
    int* hole1;
    int* simg;                           // global replay scratch for batches > kSimLds (4 arrays of C0)
    uint64_t* chg;                       // L1 keys changed this update (table patch)
    // per-update point / parent grouping hashes (cleared after use)
    uint64_t* tpk; int* tpfirst; int* tpcnt; int* tpfill; int* tppos; int* tpoff;
    uint64_t* ttk; int* ttfirst;
    uint64_t* tqk; int* tqfirst; int* tqcnt; int* tqfill; int* tqlp; int* tqoff;
    int* pslot; int* tslot; int* rslot;
    uint64_t* pkey0; uint64_t* pkey1;
    int* newlist;                        // new L0 rank -> first point
    int* glist;                          // grouped point lists
    int* rlist;                          // grouped new-L0 lists per parent
    uint64_t* T;                         // touched L1 keys
    int* tlp;                            // their positions
    int* fail;
    int* F;                              // failing touched entries (L1 positions)
    int* Foff;
    int* L0e;                            // planarity erase list (L0 positions)
    // ICP table
    Slot* tab;
    uint32_t tabl;
    unsigned long long* st;              // diagnostic phase clocks (LO_DM_STAMPS=1), else null
    float* prm;                          // this update's parameters: sensor xyz, radius^2, pose (from scan) [16]
    int* prm_n;                          // [0] point count, [1] 1 = points from the context's filtered scan
};
// diagnostic: cycles of the phase that just ended, summed over updates (read by nothing but the destroy report)
#define DM_ST(k)                                                                                    \
    do {                                                                                            \
        if (M.st) {                                                                                 \
            __syncthreads();                                                                        \
            if (threadIdx.x == 0) {                                                                 \
                const unsigned long long t_ = __builtin_amdgcn_s_memtime();                         \
                atomicAdd(&M.st[k], t_ - st_t0);                                                    \
                st_t0 = t_;                                                                         \
            }                                                                                       \
        }                                                                                           \
    } while (0)

// ---------------------------------------------------------------------------------------------- hashing
__device__ __forceinline__ uint32_t h64(uint64_t k, uint32_t l) { return static_cast<uint32_t>((k * 0x9E3779B97F4A7C15ull) >> (64 - l)); }

__device__ __forceinline__ unsigned long long* ull(uint64_t* p) { return reinterpret_cast<unsigned long long*>(p); }

// find key -> value (index tables: tombstones probed past)
__device__ int idx_find(const uint64_t* keys, const int* vals, uint32_t l, uint64_t key) {
    const uint32_t mask = (1u << l) - 1u;
    uint32_t h = h64(key, l);
    for (uint32_t p = 0; p <= mask; ++p) {
        const uint64_t k = keys[h];
        if (k == key) return vals[h];
        if (k == kEmpty) return -1;
        h = (h + 1u) & mask;
    }
    return -1;
}
// N lookups in lockstep: their probes (and the value loads) are in flight together
template <int N>
__device__ void idx_find_n(const uint64_t* keys, const int* vals, uint32_t l, const uint64_t (&key)[N],
                           const bool (&act)[N], int (&out)[N]) {
    const uint32_t mask = (1u << l) - 1u;
    uint32_t h[N];
    bool live[N], hit[N];
#pragma unroll
    for (int u = 0; u < N; ++u) { h[u] = h64(key[u], l); live[u] = act[u]; hit[u] = false; out[u] = -1; }
    for (uint32_t p = 0; p <= mask; ++p) {
        uint64_t k[N];
#pragma unroll
        for (int u = 0; u < N; ++u) k[u] = live[u] ? keys[h[u]] : kEmpty;
        bool any = false;
#pragma unroll
        for (int u = 0; u < N; ++u) {
            if (!live[u]) continue;
            if (k[u] == key[u]) { hit[u] = true; live[u] = false; }
            else if (k[u] == kEmpty) live[u] = false;
            else { h[u] = (h[u] + 1u) & mask; any = true; }
        }
        if (!any) break;
    }
#pragma unroll
    for (int u = 0; u < N; ++u) if (hit[u]) out[u] = vals[h[u]];
}
__device__ int idx_slot(const uint64_t* keys, uint32_t l, uint64_t key) {
    const uint32_t mask = (1u << l) - 1u;
    uint32_t h = h64(key, l);
    for (uint32_t p = 0; p <= mask; ++p) {
        const uint64_t k = keys[h];
        if (k == key) return static_cast<int>(h);
        if (k == kEmpty) return -1;
        h = (h + 1u) & mask;
    }
    return -1;
}
// insert a key known to be absent (CAS on the first empty slot)
__device__ void idx_insert(uint64_t* keys, int* vals, uint32_t l, uint64_t key, int val) {
    const uint32_t mask = (1u << l) - 1u;
    uint32_t h = h64(key, l);
    for (uint32_t p = 0; p <= mask;) {
        const unsigned long long prev = atomicCAS(ull(&keys[h]), static_cast<unsigned long long>(kEmpty),
                                                  static_cast<unsigned long long>(key));
        if (prev == kEmpty) { vals[h] = val; return; }
        h = (h + 1u) & mask;
        ++p;
    }
}
// group hash: insert-or-find, returns the slot
__device__ int grp_insert(uint64_t* keys, uint32_t l, uint64_t key) {
    const uint32_t mask = (1u << l) - 1u;
    uint32_t h = h64(key, l);
    for (uint32_t p = 0; p <= mask;) {
        const uint64_t k = keys[h];
        if (k == key) return static_cast<int>(h);
        if (k == kEmpty) {
            const unsigned long long prev = atomicCAS(ull(&keys[h]), static_cast<unsigned long long>(kEmpty),
                                                      static_cast<unsigned long long>(key));
            if (prev == kEmpty || prev == key) return static_cast<int>(h);
            continue;                                    // taken by another key: look at it again
        }
        h = (h + 1u) & mask;
        ++p;
    }
    return -1;
}

// ICP table (lookup_surfel's layout and probe): upsert / erase of one L1 voxel's surfel
__device__ void tab_set(Slot* tab, uint32_t l, uint64_t key, bool present, const float* n, const float* c, int* tomb) {
    const uint32_t mask = (1u << l) - 1u;
    uint32_t h = hash_slot(key, l);
    for (uint32_t p = 0; p <= mask;) {
        unsigned long long* kp = ull(&tab[h].key);
        const unsigned long long k = __hip_atomic_load(kp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == key) {
            if (!present) {
                if (atomicCAS(kp, k, static_cast<unsigned long long>(kTombKey)) == k) atomicAdd(tomb, 1);
            } else {
                for (int a = 0; a < 3; ++a) { tab[h].n[a] = n[a]; tab[h].c[a] = c[a]; }
            }
            return;
        }
        if (k == kEmptyKey) {
            if (!present) return;
            const unsigned long long prev = atomicCAS(kp, static_cast<unsigned long long>(kEmptyKey),
                                                      static_cast<unsigned long long>(key));
            if (prev == kEmptyKey) {
                for (int a = 0; a < 3; ++a) { tab[h].n[a] = n[a]; tab[h].c[a] = c[a]; }
                return;
            }
            continue;
        }
        h = (h + 1u) & mask;
        ++p;
    }
}

// point count: the host's, or the device filter's (read here, so a keyframe needs no host sync); beyond the map's
// max_points it is clipped and flagged
__device__ __forceinline__ int point_count(const DM& M, int n, const int* dn) {
    const int v = dn ? *dn : n;
    if (v > M.NP) { atomicOr(&M.cnt[C_ERR], E_CAP0); return M.NP; }
    return v < 0 ? 0 : v;
}

// ---------------------------------------------------------------------------------------------- keys
__device__ __forceinline__ bool key_ok(float f) { return f >= -1048576.0f && f < 1048576.0f; }
__device__ __forceinline__ int unpack(uint64_t k, int a) { return static_cast<int>((k >> (21 * a)) & 0x1FFFFF) - (1 << 20); }
// VoxelMap::GetParentKey (:60-67): integer floor division by the factor
__device__ __forceinline__ uint64_t parent_key(uint64_t k, int f) {
    int v[3];
    for (int a = 0; a < 3; ++a) {
        const int x = unpack(k, a);
        v[a] = x >= 0 ? x / f : (x - (f - 1)) / f;
    }
    return pack_key(v[0], v[1], v[2]);
}

// ---------------------------------------------------------------------------------------------- block primitives
// exclusive scan of one int per thread over a kOrch-thread workgroup; *total = the block's sum
__device__ int block_scan(int v, int* s_w, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    if (threadIdx.x < 64) {
        int t = threadIdx.x < (kOrch >> 6) ? s_w[threadIdx.x] : 0;
        int u = t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(u, o, 64);
            if (lane >= o) u += y;
        }
        if (threadIdx.x < (kOrch >> 6)) s_w[32 + threadIdx.x] = u - t;
        if (threadIdx.x == (kOrch >> 6) - 1) s_w[31] = u;
    }
    __syncthreads();
    const int r = s_w[32 + w] + x - v;
    *total = s_w[31];
    __syncthreads();
    return r;
}

// Ordered compaction inside one workgroup: for i < n in order, out[rank] = i where pred(i); returns the count.
template <class Pred>
__device__ int block_compact(int n, int* out, int* s_w, Pred pred) {
    int base = 0;
    for (int b = 0; b < n; b += kOrch) {
        const int i = b + static_cast<int>(threadIdx.x);
        const int f = (i < n && pred(i)) ? 1 : 0;
        int tot;
        const int r = block_scan(f, s_w, &tot);
        if (f) out[base + r] = i;
        base += tot;
    }
    return base;
}

// Replays a batch of erase-by-key operations on an insertion-ordered container of n elements (unordered_dense's
// do_erase: the last element moves into the hole) on positions only.  list = the erased elements' positions at the
// start of the batch, in erase order (distinct).  Afterwards, for every erased position e < n - q, hole[e] = the
// original position of the element that ends there.  tc / tp: q ints each (content of the tail positions
// [n - q, n) and position of the tail elements), initialised by the caller to the identity.  One lane.
__device__ void erase_sim(int n, const int* list, int q, int* tc, int* tp, int* hole) {
    const int m = n - q;
    int s = n;
    for (int k0 = 0; k0 < q; k0 += 8) {
        int ev[8];                                         // the list does not depend on the replay: read ahead
#pragma unroll
        for (int u = 0; u < 8; ++u) ev[u] = k0 + u < q ? list[k0 + u] : 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (k0 + u >= q) break;
            const int e = ev[u];
            const int L = s - 1;
            const int x = tc[L - m];
            const int p = e < m ? e : tp[e - m];
            if (p != L) {
                if (p >= m) tc[p - m] = x; else hole[p] = x;
                tp[x - m] = p;
            }
            s = L;
        }
    }
}

// The same replay with every array in LDS (explicit LDS pointers: ds_* instructions, so a step's reads never wait
// for an earlier step's memory store the way flat accesses would).  The holes' contents are kept per erase step: hs[k]
// for the step that first erased position list[k] < m; a tail element moved into a hole records -(k + 1) as its
// position.  The caller copies hs out to hole[].
typedef __attribute__((address_space(3))) int lds_int;
__device__ void erase_sim_lds(int n, const lds_int* ls, int q, lds_int* tc, lds_int* tp, lds_int* hs) {
    const int m = n - q;
    int s = n;
    for (int k0 = 0; k0 < q; k0 += 8) {
        int ev[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) ev[u] = k0 + u < q ? ls[k0 + u] : 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int k = k0 + u;
            if (k >= q) break;
            const int e = ev[u];
            const int L = s - 1;
            const int x = tc[L - m];
            int slot = -1, p = 0;
            if (e < m) slot = k;
            else {
                const int v = tp[e - m];
                if (v >= 0) p = v; else slot = -v - 1;
            }
            if (slot >= 0) {                               // a hole (L >= m, so never the last position)
                hs[slot] = x;
                tp[x - m] = -(slot + 1);
            } else if (p != L) {
                tc[p - m] = x;
                tp[x - m] = p;
            }
            s = L;
        }
    }
}

// ---------------------------------------------------------------------------------------------- container moves
__device__ void l0_move(const DM& M, int src, int dst) {
    M.k0[dst] = M.k0[src];
    for (int a = 0; a < 3; ++a) M.c0[3 * dst + a] = M.c0[3 * src + a];
    M.n0p[dst] = M.n0p[src];
}
__device__ void l1_move(const DM& M, int src, int dst) {
    M.k1[dst] = M.k1[src];
    for (int q = 0; q < kKids; ++q) M.kids[static_cast<size_t>(dst) * kKids + q] = M.kids[static_cast<size_t>(src) * kKids + q];
    M.nk[dst] = M.nk[src];
    M.has[dst] = M.has[src];
    for (int a = 0; a < 3; ++a) { M.nrm[3 * dst + a] = M.nrm[3 * src + a]; M.cen[3 * dst + a] = M.cen[3 * src + a]; }
    M.plan[dst] = M.plan[src];
    M.last[dst] = M.last[src];
}

// Both levels' erase batches (L0 list0 / q0 over n0 elements, L1 list1 / q1 over n1): replay (two lanes of
// different waves at once), then apply: erased keys leave the index (tombstone), the survivors that fill holes move
// and their index entries follow.  Block-wide; updates the counters.
__device__ void erase_batches(const DM& M, const int* list0, int q0, const int* list1, int q1, int* s_sim, int tag) {
    const int n0 = M.cnt[C_N0], n1 = M.cnt[C_N1];
    if (M.st && threadIdx.x == 0) { atomicAdd(&M.st[48 + 2 * tag], static_cast<unsigned long long>(q0));
                                    atomicAdd(&M.st[49 + 2 * tag], static_cast<unsigned long long>(q1)); }
    __shared__ int s_bad;
    if (threadIdx.x == 0) s_bad = 0;
    __syncthreads();
    for (int k = threadIdx.x; k < q0; k += kOrch) if (list0[k] < 0 || list0[k] >= n0) s_bad = 1;
    for (int k = threadIdx.x; k < q1; k += kOrch) if (list1[k] < 0 || list1[k] >= n1) s_bad = 1;
    __syncthreads();
    if (s_bad || q0 > n0 || q1 > n1) {                   // a lost key: report, leave the containers as they are
        if (threadIdx.x == 0) atomicOr(&M.cnt[C_ERR], E_LOST);
        __syncthreads();
        return;
    }
    // the replay state and the lists in LDS (a lane's dependent steps then wait on LDS, not on memory); batches
    // beyond kSimLds replay in global scratch
    const bool lds0 = q0 <= kSimLds, lds1 = q1 <= kSimLds;
    lds_int* L0s = (lds_int*)(s_sim);                                 // ls, tc, tp, hs per level (addrspacecast)
    lds_int* L1s = L0s + 4 * kSimLds;
    for (int t = threadIdx.x; t < q0; t += kOrch) {
        if (lds0) { L0s[t] = list0[t]; L0s[kSimLds + t] = n0 - q0 + t; L0s[2 * kSimLds + t] = n0 - q0 + t; }
        else { M.simg[t] = n0 - q0 + t; M.simg[M.C0 + t] = n0 - q0 + t; }
    }
    for (int t = threadIdx.x; t < q1; t += kOrch) {
        if (lds1) { L1s[t] = list1[t]; L1s[kSimLds + t] = n1 - q1 + t; L1s[2 * kSimLds + t] = n1 - q1 + t; }
        else { M.simg[2 * M.C0 + t] = n1 - q1 + t; M.simg[3 * M.C0 + t] = n1 - q1 + t; }
    }
    __syncthreads();
    if (threadIdx.x == 0 && q0 > 0) {
        if (lds0) erase_sim_lds(n0, L0s, q0, L0s + kSimLds, L0s + 2 * kSimLds, L0s + 3 * kSimLds);
        else erase_sim(n0, list0, q0, M.simg, M.simg + M.C0, M.hole0);
    }
    if (threadIdx.x == 64 && q1 > 0) {
        if (lds1) erase_sim_lds(n1, L1s, q1, L1s + kSimLds, L1s + 2 * kSimLds, L1s + 3 * kSimLds);
        else erase_sim(n1, list1, q1, M.simg + 2 * M.C0, M.simg + 3 * M.C0, M.hole1);
    }
    __syncthreads();
    const int m0 = n0 - q0, m1 = n1 - q1;
    if (lds0) for (int k = threadIdx.x; k < q0; k += kOrch) { if (L0s[k] < m0) M.hole0[L0s[k]] = L0s[3 * kSimLds + k]; }
    if (lds1) for (int k = threadIdx.x; k < q1; k += kOrch) { if (L1s[k] < m1) M.hole1[L1s[k]] = L1s[3 * kSimLds + k]; }
    __syncthreads();
    // tombstones first (the erased keys), then the moves: a moved key's index entry is found by key, and its new
    // position is an erased element's -- the two sets of keys are disjoint
    for (int k = threadIdx.x; k < q0; k += kOrch) {
        const int s = idx_slot(M.i0k, M.h0l, M.k0[list0[k]]);
        if (s >= 0) M.i0k[s] = kTomb;
    }
    for (int k = threadIdx.x; k < q1; k += kOrch) {
        const int s = idx_slot(M.i1k, M.h1l, M.k1[list1[k]]);
        if (s >= 0) M.i1k[s] = kTomb;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < q0; k += kOrch) {
        const int e = list0[k];
        if (e >= m0) continue;
        const int src = M.hole0[e];
        l0_move(M, src, e);
        const int s = idx_slot(M.i0k, M.h0l, M.k0[e]);
        if (s >= 0) M.i0v[s] = e;
    }
    for (int k = threadIdx.x; k < q1; k += kOrch) {
        const int e = list1[k];
        if (e >= m1) continue;
        const int src = M.hole1[e];
        l1_move(M, src, e);
        const int s = idx_slot(M.i1k, M.h1l, M.k1[e]);
        if (s >= 0) M.i1v[s] = e;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        M.cnt[C_N0] = m0;
        M.cnt[C_N1] = m1;
        M.cnt[C_TOMB0] += q0;
        M.cnt[C_TOMB1] += q1;
        if (4 * M.cnt[C_TOMB0] > (1 << M.h0l)) M.cnt[C_REBUILD] |= R_I0;   // the next rebuild pass renews them
        if (4 * M.cnt[C_TOMB1] > (1 << M.h1l)) M.cnt[C_REBUILD] |= R_I1;
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------------------------- kernels
// world points from a device scan: util::transform_point_cloud's order (lo_math.h transform_points)
__global__ __launch_bounds__(kPar) void k_dm_world(DM M, const float* in, const int* dn, float* out) {
    if (M.prm_n[1] != 1) return;                         // host-given points: already in place
    const int n = point_count(M, 0, dn);
    if (blockIdx.x == 0 && threadIdx.x == 0) M.prm_n[0] = n;
    float T[12];
    for (int k = 0; k < 12; ++k) T[k] = M.prm[4 + k];
    for (int i = blockIdx.x * kPar + threadIdx.x; i < n; i += gridDim.x * kPar) {
        const float x = in[3 * i], y = in[3 * i + 1], z = in[3 * i + 2];
        for (int r = 0; r < 3; ++r)
            out[3 * i + r] = ((T[4 * r] * x + T[4 * r + 1] * y) + T[4 * r + 2] * z) + T[4 * r + 3] * 1.0f;
    }
}
struct DmParams { float v[16]; int n, from_scan; };
__global__ void k_dm_setprm(DM M, DmParams P) {
    if (threadIdx.x < 16) M.prm[threadIdx.x] = P.v[threadIdx.x];
    if (threadIdx.x == 0) { M.prm_n[0] = P.n; M.prm_n[1] = P.from_scan; }
}

// prune mark (:146-157): dist^2 = (c - s).squaredNorm() > radius^2 in fp32; per-workgroup counts
__device__ __forceinline__ void prune_range(int n0, int b, int* lo, int* hi) {
    const int ch = (n0 + kPruneBlocks - 1) / kPruneBlocks;
    *lo = min(n0, b * ch);
    *hi = min(n0, *lo + ch);
}
// (an empty device-filtered cloud prunes nothing: UpdateVoxelMap returns first, :135-137)
__device__ __forceinline__ int prune_n0(const DM& M, const int* dn) { return (dn && *dn <= 0) ? 0 : M.cnt[C_N0]; }
__global__ __launch_bounds__(kPar) void k_dm_prune_mark(DM M, const int* dn) {
    __shared__ int s_c;
    const float sx = M.prm[0], sy = M.prm[1], sz = M.prm[2], rsq = M.prm[3];
    if (blockIdx.x == 0 && threadIdx.x == 0) M.cnt[C_REBUILD] = 0;        // the previous update's rebuild ran
    if (threadIdx.x == 0) s_c = 0;
    __syncthreads();
    int lo, hi;
    prune_range(prune_n0(M, dn), blockIdx.x, &lo, &hi);
    int c = 0;
    for (int i = lo + threadIdx.x; i < hi; i += kPar) {
        const float d0 = M.c0[3 * i] - sx, d1 = M.c0[3 * i + 1] - sy, d2 = M.c0[3 * i + 2] - sz;
        const float e0 = d0 * d0, e1 = d1 * d1, e2 = d2 * d2;
        const int f = (e0 + (e1 + e2) > rsq) ? 1 : 0;
        M.flag[i] = f;
        c += f;
    }
    atomicAdd(&s_c, c);
    __syncthreads();
    if (threadIdx.x == 0) M.blkcnt[blockIdx.x] = s_c;
}
// ordered compaction of the marks: D = doomed positions in L0 order
__global__ __launch_bounds__(kPar) void k_dm_prune_compact(DM M, const int* dn) {
    __shared__ int s_base, s_w[kPar / 64 + 1];
    const int b = blockIdx.x;
    if (threadIdx.x == 0) s_base = 0;
    __syncthreads();
    int part = 0;
    for (int j = threadIdx.x; j < b; j += kPar) part += M.blkcnt[j];
    atomicAdd(&s_base, part);
    __syncthreads();
    int lo, hi;
    prune_range(prune_n0(M, dn), b, &lo, &hi);
    int base = s_base;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int t = lo; t < hi; t += kPar) {
        const int i = t + threadIdx.x;
        const int f = i < hi ? M.flag[i] : 0;
        const uint64_t bal = __ballot(f);
        const int r_in = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) s_w[w] = __popcll(bal);
        __syncthreads();
        int off = 0, tot = 0;
        for (int q = 0; q < kPar / 64; ++q) { if (q < w) off += s_w[q]; tot += s_w[q]; }
        if (f) M.D[base + off + r_in] = i;
        base += tot;
        __syncthreads();
    }
    if (b == kPruneBlocks - 1 && threadIdx.x == 0) M.cnt[C_Q] = base;
}

// UnregisterFromParent (:77-97) for the doomed in L0 order, then the L0 erases in that order and the L1 erases in the
// order the voxels emptied
__global__ __launch_bounds__(kOrch) void k_dm_unregister(DM M) {
    unsigned long long st_t0 = M.st ? __builtin_amdgcn_s_memtime() : 0ull;
    __shared__ int s_w[64];
    __shared__ int s_sim[8 * kSimLds];
    const int q = M.cnt[C_Q];
    if (threadIdx.x == 0) M.cnt[C_NCHG] = 0;
    for (int j = threadIdx.x; j < q; j += kOrch) {
        M.emptied[j] = -1;
        const int lp = idx_find(M.i1k, M.i1v, M.h1l, parent_key(M.k0[M.D[j]], M.factor));
        if (lp < 0) { atomicOr(&M.cnt[C_ERR], E_LOST); continue; }
        const int k = atomicAdd(&M.ucnt[lp], 1);
        if (k < kKids) M.ulist[static_cast<size_t>(lp) * kKids + k] = j;
        else atomicOr(&M.cnt[C_ERR], E_KIDS);
    }
    DM_ST(30);
    // one lane per parent (the lane of its first doomed child in list order): its children set's erases in L0 order
    for (int j = threadIdx.x; j < q; j += kOrch) {
        M.flag[j] = -1;                                    // the parent position when j leads it
        const int lp = idx_find(M.i1k, M.i1v, M.h1l, parent_key(M.k0[M.D[j]], M.factor));
        if (lp < 0) continue;
        const int* L = M.ulist + static_cast<size_t>(lp) * kKids;
        const int c = min(M.ucnt[lp], kKids);
        int first = L[0];
        for (int t = 1; t < c; ++t) first = min(first, L[t]);
        if (first == j) M.flag[j] = lp;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < q; j += kOrch) {
        const int lp = M.flag[j];
        if (lp < 0) continue;
        int* L = M.ulist + static_cast<size_t>(lp) * kKids;
        const int c = min(M.ucnt[lp], kKids);
        for (int a = 1; a < c; ++a) {                      // insertion sort: list order
            const int v = L[a];
            int b = a - 1;
            while (b >= 0 && L[b] > v) { L[b + 1] = L[b]; --b; }
            L[b + 1] = v;
        }
        uint64_t* K = M.kids + static_cast<size_t>(lp) * kKids;
        int nk = M.nk[lp];
        for (int t = 0; t < c; ++t) {
            const uint64_t key = M.k0[M.D[L[t]]];
            for (int u = 0; u < nk; ++u)
                if (K[u] == key) { K[u] = K[nk - 1]; --nk; break; }
        }
        M.nk[lp] = nk;
        if (nk < 5) M.has[lp] = 0;
        if (nk == 0) M.emptied[L[c - 1]] = lp;
        M.ucnt[lp] = 0;
        M.chg[atomicAdd(&M.cnt[C_NCHG], 1)] = M.k1[lp];
    }
    __syncthreads();
    DM_ST(31);
    const int q1 = block_compact(q, M.E1, s_w, [&](int j) { return M.emptied[j] >= 0; });
    for (int t = threadIdx.x; t < q1; t += kOrch) M.E1[t] = M.emptied[M.E1[t]];
    __syncthreads();
    DM_ST(32);
    erase_batches(M, M.D, q, M.E1, q1, s_sim, 0);
    DM_ST(33);
}

// per point: L0 / L1 keys (PointToVoxelKey, :50-58) and the grouping hashes (first occurrence, size)
__device__ void dm_keys_one(const DM& M, const float* pts, int i) {
    float f0[3], f1[3];
    bool ok = true;
    for (int a = 0; a < 3; ++a) {
        const float p = pts[3 * i + a];
        f0[a] = floorf(p / M.voxel);
        f1[a] = floorf(p / M.l1scale);
        ok = ok && key_ok(f0[a]) && key_ok(f1[a]);
    }
    if (!ok) { atomicOr(&M.cnt[C_ERR], E_KEY); M.pslot[i] = M.tslot[i] = -1; return; }
    const uint64_t a0 = pack_key(static_cast<int>(f0[0]), static_cast<int>(f0[1]), static_cast<int>(f0[2]));
    const uint64_t a1 = pack_key(static_cast<int>(f1[0]), static_cast<int>(f1[1]), static_cast<int>(f1[2]));
    M.pkey0[i] = a0;
    M.pkey1[i] = a1;
    const int s0 = grp_insert(M.tpk, M.hpl, a0);
    const int s1 = grp_insert(M.ttk, M.hpl, a1);
    M.pslot[i] = s0;
    M.tslot[i] = s1;
    if (s0 < 0 || s1 < 0) { atomicOr(&M.cnt[C_ERR], E_CAP0); M.pslot[i] = M.tslot[i] = -1; return; }
    atomicMin(&M.tpfirst[s0], i);
    atomicAdd(&M.tpcnt[s0], 1);
    atomicMin(&M.ttfirst[s1], i);
}
__global__ __launch_bounds__(kPar) void k_dm_keys(DM M, const float* pts, int n_host, const int* dn) {
    const int n = point_count(M, n_host, dn);
    for (int i = blockIdx.x * kPar + threadIdx.x; i < n; i += gridDim.x * kPar) dm_keys_one(M, pts, i);
}

// AddPoint for every point in order (:99-120, :171-181) and the touched L1 set, as a pipeline of launches: the
// per-item work runs on many CUs (a single workgroup was bound by one CU's gather rate), and the order-defining ranks
// come from ordered passes: kChunk workgroups each own a contiguous chunk of the items, count (a_*), one workgroup
// scans the chunk counts (k_dm_scan3), and every chunk then ranks its items with a block-local scan (b_*).
#define FOR_U _Pragma("unroll") for (int u = 0; u < kU; ++u)
__device__ __forceinline__ void chunk_range(int n, int b, int G, int* lo, int* hi) {
    const int ch = (n + G - 1) / G;
    *lo = min(n, b * ch);
    *hi = min(n, *lo + ch);
}
// exclusive scan over a kPar-thread workgroup
__device__ int scan_par(int v, int* s_w, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int q = 0; q < kPar / 64; ++q) { if (q < w) off += s_w[q]; tot += s_w[q]; }
    __syncthreads();
    *total = tot;
    return off + x - v;
}
__device__ __forceinline__ int npts(const DM& M, int n_host, const int* dn) { return dn ? min(*dn, M.NP) : n_host; }

// (1) per point: the existing voxel of its group (looked up at the group's first point); chunk counts of new groups,
// group sizes and touched-key first occurrences
__global__ __launch_bounds__(kPar) void k_dm_a_count(DM M, int n_host, const int* dn) {
    __shared__ int s_c[3];
    const int n = npts(M, n_host, dn);
    if (threadIdx.x < 3) s_c[threadIdx.x] = 0;
    __syncthreads();
    int lo, hi;
    chunk_range(n, blockIdx.x, gridDim.x, &lo, &hi);
    int c0 = 0, c1 = 0, c2 = 0;
    for (int i = lo + threadIdx.x; i < hi; i += kPar) {
        const int sl = M.pslot[i], s1 = M.tslot[i];
        if (sl >= 0 && M.tpfirst[sl] == i) {
            const int pos = idx_find(M.i0k, M.i0v, M.h0l, M.pkey0[i]);
            M.tppos[sl] = pos;
            c0 += pos < 0 ? 1 : 0;
            c1 += M.tpcnt[sl];
        }
        if (s1 >= 0 && M.ttfirst[s1] == i) ++c2;
    }
    atomicAdd(&s_c[0], c0);
    atomicAdd(&s_c[1], c1);
    atomicAdd(&s_c[2], c2);
    __syncthreads();
    if (threadIdx.x < 3) M.bc[threadIdx.x * kChunk + blockIdx.x] = s_c[threadIdx.x];
}
// chunk offsets of three counts (stage 1: new L0 / group lists / touched; stage 2: new L1 / child lists)
__global__ __launch_bounds__(kOrch) void k_dm_scan3(DM M, int stage) {
    __shared__ int s_w[64];
    const int t = threadIdx.x;
    int tot[3];
    for (int k = 0; k < 3; ++k) {
        const int v = t < kChunk ? M.bc[k * kChunk + t] : 0;
        const int r = block_scan(v, s_w, &tot[k]);
        if (t < kChunk) M.bo[k * kChunk + t] = r;
    }
    if (t != 0) return;
    if (stage == 1) {
        const int n0 = M.cnt[C_N0];
        M.cnt[C_NNEW] = tot[0];
        M.cnt[C_NT] = tot[2];
        M.cnt[C_ABORT] = 0;
        if (n0 + tot[0] > M.C0) { atomicOr(&M.cnt[C_ERR], E_CAP0); M.cnt[C_ABORT] = 1; M.cnt[C_NT] = 0; }
    } else {
        M.cnt[C_NL1] = tot[0];
        if (M.cnt[C_N1] + tot[0] > M.C1) { atomicOr(&M.cnt[C_ERR], E_CAP1); M.cnt[C_ABORT] = 2; M.cnt[C_NT] = 0; }
    }
}
// (2) ranks: new L0 voxels appended in first-occurrence order, group list offsets, the touched list
__global__ __launch_bounds__(kPar) void k_dm_a_rank(DM M, int n_host, const int* dn) {
    __shared__ int s_w[kPar / 64];
    if (M.cnt[C_ABORT]) return;
    const int n = npts(M, n_host, dn);
    const int n0 = M.cnt[C_N0];
    int lo, hi;
    chunk_range(n, blockIdx.x, gridDim.x, &lo, &hi);
    int b0 = M.bo[blockIdx.x], b1 = M.bo[kChunk + blockIdx.x], b2 = M.bo[2 * kChunk + blockIdx.x];
    for (int t = lo; t < hi; t += kPar) {
        const int i = t + threadIdx.x;
        int sl = -1, v0 = 0, v1 = 0, v2 = 0;
        if (i < hi) {
            sl = M.pslot[i];
            const int s1 = M.tslot[i];
            if (sl >= 0 && M.tpfirst[sl] == i) { v0 = M.tppos[sl] < 0 ? 1 : 0; v1 = M.tpcnt[sl]; }
            v2 = (s1 >= 0 && M.ttfirst[s1] == i) ? 1 : 0;
        }
        int t0, t1, t2;
        const int r0 = scan_par(v0, s_w, &t0);
        const int r1 = scan_par(v1, s_w, &t1);
        const int r2 = scan_par(v2, s_w, &t2);
        if (v0) {
            const int pos = n0 + b0 + r0;
            M.newlist[b0 + r0] = i;
            M.tppos[sl] = pos;
            M.k0[pos] = M.pkey0[i];
            M.n0p[pos] = 0;
        }
        if (v1) M.tpoff[sl] = b1 + r1;
        if (v2) M.T[b2 + r2] = M.pkey1[i];
        b0 += t0; b1 += t1; b2 += t2;
    }
}
// (3) the groups' point lists
__global__ __launch_bounds__(kPar) void k_dm_a_fill(DM M, int n_host, const int* dn) {
    if (M.cnt[C_ABORT]) return;
    const int n = npts(M, n_host, dn);
    for (int i = blockIdx.x * kPar + threadIdx.x; i < n; i += gridDim.x * kPar) {
        const int sl = M.pslot[i];
        if (sl >= 0) M.glist[M.tpoff[sl] + atomicAdd(&M.tpfill[sl], 1)] = i;
    }
}
// (4) running mean per voxel over its points in point order (fp32, (c n + p) / (n + 1)); one lane per group
__global__ __launch_bounds__(kPar) void k_dm_a_mean(DM M, const float* pts, int n_host, const int* dn) {
    if (M.cnt[C_ABORT]) return;
    const int n = npts(M, n_host, dn);
    for (int i = blockIdx.x * kPar + threadIdx.x; i < n; i += gridDim.x * kPar) {
        const int sl = M.pslot[i];
        if (sl < 0 || M.tpfirst[sl] != i) continue;
        int* L = M.glist + M.tpoff[sl];
        const int c = M.tpcnt[sl];
        for (int a2 = 1; a2 < c; ++a2) {
            const int v = L[a2];
            int q = a2 - 1;
            while (q >= 0 && L[q] > v) { L[q + 1] = L[q]; --q; }
            L[q + 1] = v;
        }
        const int pos = M.tppos[sl];
        float cx = M.c0[3 * pos], cy = M.c0[3 * pos + 1], cz = M.c0[3 * pos + 2];
        int np = M.n0p[pos];
        for (int t = 0; t < c; ++t) {
            const float* p = pts + 3 * L[t];
            if (np == 0) {
                cx = p[0]; cy = p[1]; cz = p[2];
                np = 1;
            } else {
                const float nf = static_cast<float>(np), n1f = static_cast<float>(np + 1);
                cx = (cx * nf + p[0]) / n1f;
                cy = (cy * nf + p[1]) / n1f;
                cz = (cz * nf + p[2]) / n1f;
                ++np;
            }
        }
        M.c0[3 * pos] = cx; M.c0[3 * pos + 1] = cy; M.c0[3 * pos + 2] = cz;
        M.n0p[pos] = np;
    }
}
// (5) RegisterToParent (:69-75) for the new L0 voxels in creation order: group them by parent
__global__ __launch_bounds__(kPar) void k_dm_r_group(DM M) {
    if (M.cnt[C_ABORT]) return;
    const int nnew = M.cnt[C_NNEW], n0 = M.cnt[C_N0];
    for (int r = blockIdx.x * kPar + threadIdx.x; r < nnew; r += gridDim.x * kPar) {
        const int s = grp_insert(M.tqk, M.hpl, parent_key(M.k0[n0 + r], M.factor));   // capacity >= 2 max_points
        M.rslot[r] = s;
        atomicMin(&M.tqfirst[s], r);
        atomicAdd(&M.tqcnt[s], 1);
    }
}
// (6) each parent (at its first new child): existing L1 voxel or not; chunk counts of new L1s and child lists
__global__ __launch_bounds__(kPar) void k_dm_r_count(DM M) {
    __shared__ int s_c[2];
    if (M.cnt[C_ABORT]) return;
    const int nnew = M.cnt[C_NNEW];
    if (threadIdx.x < 2) s_c[threadIdx.x] = 0;
    __syncthreads();
    int lo, hi;
    chunk_range(nnew, blockIdx.x, gridDim.x, &lo, &hi);
    int c0 = 0, c1 = 0;
    for (int r = lo + threadIdx.x; r < hi; r += kPar) {
        const int s = M.rslot[r];
        if (M.tqfirst[s] != r) continue;
        const int lp = idx_find(M.i1k, M.i1v, M.h1l, M.tqk[s]);
        M.tqlp[s] = lp;
        c0 += lp < 0 ? 1 : 0;
        c1 += M.tqcnt[s];
    }
    atomicAdd(&s_c[0], c0);
    atomicAdd(&s_c[1], c1);
    __syncthreads();
    if (threadIdx.x < 3) M.bc[threadIdx.x * kChunk + blockIdx.x] = threadIdx.x < 2 ? s_c[threadIdx.x] : 0;
}
// (7) new L1 voxels appended in first-child order; child-list offsets
__global__ __launch_bounds__(kPar) void k_dm_r_rank(DM M) {
    __shared__ int s_w[kPar / 64];
    if (M.cnt[C_ABORT]) return;
    const int nnew = M.cnt[C_NNEW], n1 = M.cnt[C_N1];
    int lo, hi;
    chunk_range(nnew, blockIdx.x, gridDim.x, &lo, &hi);
    int b0 = M.bo[blockIdx.x], b1 = M.bo[kChunk + blockIdx.x];
    for (int t = lo; t < hi; t += kPar) {
        const int r = t + threadIdx.x;
        int s = 0, v0 = 0, v1 = 0;
        if (r < hi) {
            s = M.rslot[r];
            if (M.tqfirst[s] == r) { v0 = M.tqlp[s] < 0 ? 1 : 0; v1 = M.tqcnt[s]; }
        }
        int t0, t1;
        const int r0 = scan_par(v0, s_w, &t0);
        const int r1 = scan_par(v1, s_w, &t1);
        if (v0) {
            const int lp = n1 + b0 + r0;
            M.tqlp[s] = lp;
            M.k1[lp] = M.tqk[s];
            M.nk[lp] = 0;
            M.has[lp] = 0;
            for (int a2 = 0; a2 < 3; ++a2) { M.nrm[3 * lp + a2] = 0.0f; M.cen[3 * lp + a2] = 0.0f; }
            M.plan[lp] = 1.0f;
            M.last[lp] = 0;
        }
        if (v1) M.tqoff[s] = b1 + r1;
        b0 += t0; b1 += t1;
    }
}
__global__ __launch_bounds__(kPar) void k_dm_r_fill(DM M) {
    if (M.cnt[C_ABORT]) return;
    const int nnew = M.cnt[C_NNEW];
    for (int r = blockIdx.x * kPar + threadIdx.x; r < nnew; r += gridDim.x * kPar) {
        const int s = M.rslot[r];
        M.rlist[M.tqoff[s] + atomicAdd(&M.tqfill[s], 1)] = r;
    }
}
// (8) each parent's new children in creation order appended to its children set; index entries of the new voxels
__global__ __launch_bounds__(kPar) void k_dm_r_append(DM M) {
    if (M.cnt[C_ABORT]) return;
    const int nnew = M.cnt[C_NNEW], n0 = M.cnt[C_N0], n1 = M.cnt[C_N1];
    for (int r = blockIdx.x * kPar + threadIdx.x; r < nnew; r += gridDim.x * kPar) {
        idx_insert(M.i0k, M.i0v, M.h0l, M.k0[n0 + r], n0 + r);
        const int s = M.rslot[r];
        if (M.tqfirst[s] != r) continue;
        int* L = M.rlist + M.tqoff[s];
        const int c = M.tqcnt[s];
        for (int a2 = 1; a2 < c; ++a2) {
            const int v = L[a2];
            int q = a2 - 1;
            while (q >= 0 && L[q] > v) { L[q + 1] = L[q]; --q; }
            L[q + 1] = v;
        }
        const int lp = M.tqlp[s];
        if (lp >= n1) idx_insert(M.i1k, M.i1v, M.h1l, M.tqk[s], lp);
        const int nk = M.nk[lp];
        if (nk + c > kKids) { atomicOr(&M.cnt[C_ERR], E_KIDS); continue; }
        for (int t = 0; t < c; ++t) M.kids[static_cast<size_t>(lp) * kKids + nk + t] = M.k0[n0 + L[t]];
        M.nk[lp] = nk + c;
    }
}
// (9) the grouping hashes return to empty (only the slots this update used); the new counts
__global__ __launch_bounds__(kPar) void k_dm_a_done(DM M, int n_host, const int* dn) {
    const int n = npts(M, n_host, dn);
    const int ab = M.cnt[C_ABORT];
    const int nreg = ab == 1 ? 0 : M.cnt[C_NNEW];
    const int stride = gridDim.x * kPar, t0 = blockIdx.x * kPar + threadIdx.x;
    for (int i = t0; i < n; i += stride) {
        const int sl = M.pslot[i], s1 = M.tslot[i];
        if (sl >= 0) { M.tpk[sl] = kEmpty; M.tpfirst[sl] = INT_MAX; M.tpcnt[sl] = 0; M.tpfill[sl] = 0; }
        if (s1 >= 0) { M.ttk[s1] = kEmpty; M.ttfirst[s1] = INT_MAX; }
    }
    for (int r = t0; r < nreg; r += stride) {
        const int s = M.rslot[r];
        M.tqk[s] = kEmpty; M.tqfirst[s] = INT_MAX; M.tqcnt[s] = 0; M.tqfill[s] = 0;
    }
    if (t0 == 0 && !ab) {
        M.cnt[C_N0] += M.cnt[C_NNEW];
        M.cnt[C_N1] += M.cnt[C_NL1];
    }
}

// the touched voxels' surfel decisions and refits (:183-261), all in parallel: each reads only its own children
__device__ void dm_touched_one(const DM& M, int t, float* cs) {
    M.fail[t] = 0;
    const int lp = idx_find(M.i1k, M.i1v, M.h1l, M.T[t]);
    M.tlp[t] = lp;
    if (lp < 0) return;                                    // cannot happen: every touched key registered above
    if (!M.surfels) return;                                // UpdateVoxelMap returns before the surfel pass
    const int cnt = M.nk[lp];
    if (cnt < 5) { M.has[lp] = 0; return; }
    if (M.has[lp] && M.last[lp] == cnt) return;
    int m = 0;
    for (int q0 = 0; q0 < cnt; q0 += 9) {                 // the children's lookups nine at a time
        uint64_t ck[9];
        bool act[9];
        int pos[9];
#pragma unroll
        for (int u = 0; u < 9; ++u) {
            act[u] = q0 + u < cnt;
            ck[u] = act[u] ? M.kids[static_cast<size_t>(lp) * kKids + q0 + u] : 0;
        }
        idx_find_n<9>(M.i0k, M.i0v, M.h0l, ck, act, pos);
#pragma unroll
        for (int u = 0; u < 9; ++u) {
            if (!act[u] || pos[u] < 0) continue;
            for (int a = 0; a < 3; ++a) cs[3 * m + a] = M.c0[3 * pos[u] + a];
            ++m;
        }
    }
    if (m < 3) { M.has[lp] = 0; return; }
    float cen[3], U[3][3];
    const float planarity = surfel_fit(cs, m, cen, U);
    if (planarity > M.thr) { M.has[lp] = 0; M.fail[t] = 1; return; }
    M.has[lp] = 1;
    for (int a = 0; a < 3; ++a) { M.nrm[3 * lp + a] = U[a][2]; M.cen[3 * lp + a] = cen[a]; }
    M.plan[lp] = planarity;
    M.last[lp] = cnt;
}
__global__ __launch_bounds__(64) void k_dm_touched(DM M) {       // 64-lane workgroups: the fits spread over CUs
    __shared__ float s_cs[64 * 3 * kKids];                           // each lane's child centroids (not scratch)
    const int nt = M.cnt[C_NT];
    for (int t = blockIdx.x * 64 + threadIdx.x; t < nt; t += gridDim.x * 64)
        dm_touched_one(M, t, s_cs + threadIdx.x * 3 * kKids);
}

// planarity failures in touched order: the voxel's children (child order), then the voxel; then the table patch of
// every changed key
__global__ __launch_bounds__(kOrch) void k_dm_finish(DM M) {
    unsigned long long st_t0 = M.st ? __builtin_amdgcn_s_memtime() : 0ull;
    __shared__ int s_w[64];
    __shared__ int s_sim[8 * kSimLds];
    const int nt = M.cnt[C_NT];
    const int nf = block_compact(nt, M.F, s_w, [&](int t) { return M.fail[t] != 0; });
    DM_ST(20);
    int base = 0;
    for (int b = 0; b < nf; b += kOrch) {
        const int f = b + static_cast<int>(threadIdx.x);
        const int v = f < nf ? M.nk[M.tlp[M.F[f]]] : 0;
        int tot;
        const int o = block_scan(v, s_w, &tot);
        if (f < nf) M.Foff[f] = base + o;
        base += tot;
    }
    const int q0 = base;
    DM_ST(21);
    __shared__ int s_foff[1025];
    for (int f = threadIdx.x; f < nf; f += kOrch) {
        M.E1[f] = M.tlp[M.F[f]];
        if (nf <= 1024) s_foff[f] = M.Foff[f];
    }
    if (threadIdx.x == 0 && nf <= 1024) s_foff[nf] = q0;
    __syncthreads();
    if (nf <= 1024) {
        // one lane per child (voxel by binary search over the offsets), the lookups kU at a time
        for (int b = 0; b < q0; b += kU * kOrch) {
            int k[kU], pos[kU];
            uint64_t key[kU];
            bool act[kU];
            FOR_U {
                k[u] = b + u * kOrch + threadIdx.x;
                act[u] = k[u] < q0;
                key[u] = 0;
                if (act[u]) {
                    int lo = 0, hi = nf;                   // last f with s_foff[f] <= k
                    while (hi - lo > 1) { const int mid = (lo + hi) >> 1; if (s_foff[mid] <= k[u]) lo = mid; else hi = mid; }
                    key[u] = M.kids[static_cast<size_t>(M.E1[lo]) * kKids + (k[u] - s_foff[lo])];
                }
            }
            idx_find_n<kU>(M.i0k, M.i0v, M.h0l, key, act, pos);
            FOR_U if (act[u]) M.L0e[k[u]] = pos[u];
        }
    } else {
        for (int f = threadIdx.x; f < nf; f += kOrch) {
            const int lp = M.E1[f];
            for (int c = 0; c < M.nk[lp]; ++c)
                M.L0e[M.Foff[f] + c] = idx_find(M.i0k, M.i0v, M.h0l, M.kids[static_cast<size_t>(lp) * kKids + c]);
        }
    }
    __syncthreads();
    DM_ST(22);
    erase_batches(M, M.L0e, q0, M.E1, nf, s_sim, 1);
    DM_ST(23);
    DM_ST(24);
}

// the ICP table: every changed key's final state (unregistered parents, touched voxels; erased ones are absent)
__global__ __launch_bounds__(kPar) void k_dm_table(DM M) {
    const int nc = M.cnt[C_NCHG], nt = M.cnt[C_NT];
    for (int k = blockIdx.x * kPar + threadIdx.x; k < nc + nt; k += gridDim.x * kPar) {
        const uint64_t key = k < nc ? M.chg[k] : M.T[k - nc];
        const int lp = idx_find(M.i1k, M.i1v, M.h1l, key);
        const bool present = lp >= 0 && M.has[lp];
        tab_set(M.tab, M.tabl, key, present, present ? M.nrm + 3 * lp : nullptr, present ? M.cen + 3 * lp : nullptr,
                &M.cnt[C_TTOMB]);
    }
}
__global__ void k_dm_table_check(DM M) {
    if (threadIdx.x == 0 && 4 * M.cnt[C_TTOMB] > (1 << M.tabl)) M.cnt[C_REBUILD] |= R_TAB;
}

// renewal of the tombstoned indices / table when flagged (clear pass, then insert pass)
__global__ __launch_bounds__(kPar) void k_dm_rebuild_clear(DM M) {
    const int fl = M.cnt[C_REBUILD];
    if (!fl) return;
    const size_t stride = static_cast<size_t>(gridDim.x) * kPar;
    const size_t t0 = static_cast<size_t>(blockIdx.x) * kPar + threadIdx.x;
    if (fl & R_I0) for (size_t i = t0; i < (size_t(1) << M.h0l); i += stride) M.i0k[i] = kEmpty;
    if (fl & R_I1) for (size_t i = t0; i < (size_t(1) << M.h1l); i += stride) M.i1k[i] = kEmpty;
    if (fl & R_TAB)
        for (size_t i = t0; i < (size_t(1) << M.tabl); i += stride) {
            M.tab[i].key = kEmptyKey;
            for (int a = 0; a < 3; ++a) { M.tab[i].n[a] = 0.0f; M.tab[i].c[a] = 0.0f; }
        }
}
__global__ __launch_bounds__(kPar) void k_dm_rebuild_fill(DM M) {
    const int fl = M.cnt[C_REBUILD];
    if (!fl) return;
    const int stride = gridDim.x * kPar;
    const int t0 = blockIdx.x * kPar + threadIdx.x;
    if (fl & R_I0) for (int i = t0; i < M.cnt[C_N0]; i += stride) idx_insert(M.i0k, M.i0v, M.h0l, M.k0[i], i);
    if (fl & R_I1) for (int i = t0; i < M.cnt[C_N1]; i += stride) idx_insert(M.i1k, M.i1v, M.h1l, M.k1[i], i);
    if (fl & R_TAB)
        for (int i = t0; i < M.cnt[C_N1]; i += stride)
            if (M.has[i]) tab_set(M.tab, M.tabl, M.k1[i], true, M.nrm + 3 * i, M.cen + 3 * i, nullptr);
    if (t0 == 0) {
        if (fl & R_I0) M.cnt[C_TOMB0] = 0;
        if (fl & R_I1) M.cnt[C_TOMB1] = 0;
        if (fl & R_TAB) M.cnt[C_TTOMB] = 0;
    }
}

// ---------------------------------------------------------------------------------------------- ApplyTransformAndRehash
// (:264-302) every L0 centroid moved (R c + t, Matrix3f * Vector3f) and re-keyed; the rebuilt L0 holds the keys in
// first-occurrence order, colliding voxels merged in the old order ((c1 n1 + c2 n2) / (n1 + n2)); every entry
// registers with its parent, so L1 is ordered by first child and each children set by L0 position.
__global__ __launch_bounds__(kPar) void k_dm_at_keys(DM M, DmPose T, float* tc, uint64_t* tk) {
    const int i = blockIdx.x * kPar + threadIdx.x;
    if (i >= M.cnt[C_N0]) return;
    const float* c = M.c0 + 3 * i;
    float o[3];
    for (int r = 0; r < 3; ++r)
        o[r] = dot3e(T.v[4 * r], T.v[4 * r + 1], T.v[4 * r + 2], c[0], c[1], c[2]) + T.v[4 * r + 3];
    float f[3];
    bool ok = true;
    for (int a = 0; a < 3; ++a) { tc[3 * i + a] = o[a]; f[a] = floorf(o[a] / M.voxel); ok = ok && key_ok(f[a]); }
    if (!ok) { atomicOr(&M.cnt[C_ERR], E_KEY); f[0] = f[1] = f[2] = 0.0f; }
    tk[i] = pack_key(static_cast<int>(f[0]), static_cast<int>(f[1]), static_cast<int>(f[2]));
}

__global__ __launch_bounds__(kOrch) void k_dm_at_rebuild(DM M, const float* tc, const uint64_t* tk, int* tslot,
                                                         int* tfirst, int* tcnt, int* toff, int* tfill, int* glist,
                                                         int* order, uint64_t* nk0, float* nc0, int* nn0) {
    __shared__ int s_w[64];
    const int n = M.cnt[C_N0];
    // grouping by new key (hash of capacity 2^hpl >= 2 C0 reserved in the point hashes' place)
    for (int i = threadIdx.x; i < n; i += kOrch) {
        const int s = grp_insert(M.tpk, M.h0l, tk[i]);
        tslot[i] = s;
        atomicMin(&tfirst[s], i);
        atomicAdd(&tcnt[s], 1);
    }
    __syncthreads();
    const int G = block_compact(n, order, s_w, [&](int i) { return tfirst[tslot[i]] == i; });
    int base = 0;
    for (int b = 0; b < G; b += kOrch) {
        const int g = b + static_cast<int>(threadIdx.x);
        const int v = g < G ? tcnt[tslot[order[g]]] : 0;
        int tot;
        const int o = block_scan(v, s_w, &tot);
        if (g < G) toff[tslot[order[g]]] = base + o;
        base += tot;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kOrch) glist[toff[tslot[i]] + atomicAdd(&tfill[tslot[i]], 1)] = i;
    __syncthreads();
    for (int g = threadIdx.x; g < G; g += kOrch) {
        const int s = tslot[order[g]];
        int* L = glist + toff[s];
        const int c = tcnt[s];
        for (int a = 1; a < c; ++a) {
            const int v = L[a];
            int b = a - 1;
            while (b >= 0 && L[b] > v) { L[b + 1] = L[b]; --b; }
            L[b + 1] = v;
        }
        float x = tc[3 * L[0]], y = tc[3 * L[0] + 1], z = tc[3 * L[0] + 2];
        int np = M.n0p[L[0]];
        for (int t = 1; t < c; ++t) {
            const int j = L[t];
            const float n1 = static_cast<float>(np), n2 = static_cast<float>(M.n0p[j]);
            x = (x * n1 + tc[3 * j] * n2) / (n1 + n2);
            y = (y * n1 + tc[3 * j + 1] * n2) / (n1 + n2);
            z = (z * n1 + tc[3 * j + 2] * n2) / (n1 + n2);
            np += M.n0p[j];
        }
        nk0[g] = tk[order[g]];
        nc0[3 * g] = x; nc0[3 * g + 1] = y; nc0[3 * g + 2] = z;
        nn0[g] = np;
    }
    __syncthreads();
    for (int g = threadIdx.x; g < G; g += kOrch) {
        M.k0[g] = nk0[g];
        for (int a = 0; a < 3; ++a) M.c0[3 * g + a] = nc0[3 * g + a];
        M.n0p[g] = nn0[g];
    }
    for (int i = threadIdx.x; i < n; i += kOrch) {
        const int s = tslot[i];
        M.tpk[s] = kEmpty; tfirst[s] = INT_MAX; tcnt[s] = 0; tfill[s] = 0;
    }
    __syncthreads();
    // L1 from scratch: parents in first-child order, children by L0 position
    for (int g = threadIdx.x; g < G; g += kOrch) {
        const int s = grp_insert(M.tpk, M.h0l, parent_key(M.k0[g], M.factor));
        tslot[g] = s;
        atomicMin(&tfirst[s], g);
        atomicAdd(&tcnt[s], 1);
    }
    __syncthreads();
    const int P = block_compact(G, order, s_w, [&](int g) { return tfirst[tslot[g]] == g; });
    if (P > M.C1) { if (threadIdx.x == 0) atomicOr(&M.cnt[C_ERR], E_CAP1); }
    for (int p = threadIdx.x; p < min(P, M.C1); p += kOrch) toff[tslot[order[p]]] = p;
    __syncthreads();
    for (int p = threadIdx.x; p < min(P, M.C1); p += kOrch) {
        M.k1[p] = M.tpk[tslot[order[p]]];
        M.nk[p] = 0;
        M.has[p] = 0;
        for (int a = 0; a < 3; ++a) { M.nrm[3 * p + a] = 0.0f; M.cen[3 * p + a] = 0.0f; }
        M.plan[p] = 1.0f;
        M.last[p] = 0;
    }
    __syncthreads();
    // children: each parent's L0 positions ascending (appended in any order, then sorted; ulist is free here)
    for (int g = threadIdx.x; g < G; g += kOrch) {
        const int s = tslot[g];
        const int p = toff[s];
        if (p >= M.C1) continue;
        const int k = atomicAdd(&tfill[s], 1);
        if (k < kKids) M.ulist[static_cast<size_t>(p) * kKids + k] = g;
        else atomicOr(&M.cnt[C_ERR], E_KIDS);
    }
    __syncthreads();
    for (int p = threadIdx.x; p < min(P, M.C1); p += kOrch) {
        const int s = tslot[order[p]];
        const int c = min(tfill[s], kKids);
        int* L = M.ulist + static_cast<size_t>(p) * kKids;
        for (int a = 1; a < c; ++a) {
            const int v = L[a];
            int b = a - 1;
            while (b >= 0 && L[b] > v) { L[b + 1] = L[b]; --b; }
            L[b + 1] = v;
        }
        for (int a = 0; a < c; ++a) M.kids[static_cast<size_t>(p) * kKids + a] = M.k0[L[a]];
        M.nk[p] = c;
    }
    __syncthreads();
    for (int g = threadIdx.x; g < G; g += kOrch) {
        const int s = tslot[g];
        M.tpk[s] = kEmpty; tfirst[s] = INT_MAX; tcnt[s] = 0; tfill[s] = 0;
    }
    if (threadIdx.x == 0) {
        M.cnt[C_N0] = G;
        M.cnt[C_N1] = min(P, M.C1);
    }
}

// RecomputeAllSurfels (:304-366): every L1 voxel refitted; failures only lose the surfel
__global__ __launch_bounds__(kPar) void k_dm_recompute(DM M) {
    const int lp = blockIdx.x * kPar + threadIdx.x;
    if (lp >= M.cnt[C_N1]) return;
    const int cnt = M.nk[lp];
    if (cnt < 5) { M.has[lp] = 0; return; }
    float cs[3 * kKids];
    int m = 0;
    for (int q = 0; q < cnt; ++q) {
        const int p = idx_find(M.i0k, M.i0v, M.h0l, M.kids[static_cast<size_t>(lp) * kKids + q]);
        if (p < 0) continue;
        for (int a = 0; a < 3; ++a) cs[3 * m + a] = M.c0[3 * p + a];
        ++m;
    }
    if (m < 5) { M.has[lp] = 0; return; }
    float cen[3], U[3][3];
    const float planarity = surfel_fit(cs, m, cen, U);
    if (planarity > M.thr) { M.has[lp] = 0; return; }
    M.has[lp] = 1;
    for (int a = 0; a < 3; ++a) { M.nrm[3 * lp + a] = U[a][2]; M.cen[3 * lp + a] = cen[a]; }
    M.plan[lp] = planarity;
    M.last[lp] = cnt;
}

__global__ __launch_bounds__(kPar) void k_dm_flag(DM M, int flags) {
    if (blockIdx.x == 0 && threadIdx.x == 0) M.cnt[C_REBUILD] |= flags;
}

}  // namespace dm
}  // namespace lo

// ================================================================================================== host side
using namespace lo;
using namespace lo::dm;

struct lo_devmap {
    lo_ctx* ctx = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    DM M{};
    std::vector<void*> bufs;
    float* d_in = nullptr;               // world points (host input / device transform target)
    float* at_c = nullptr;               // ApplyTransformAndRehash scratch: moved centroids, new keys, merged L0
    uint64_t* at_k = nullptr;
    uint64_t* at_nk = nullptr;
    float* at_nc = nullptr;
    int* at_nn = nullptr;
    uint64_t tab_gen = 0;
    hipGraphExec_t gexec = nullptr;      // the captured update pipeline and what it was captured with
    Slot* g_tab = nullptr;
    uint32_t g_tabl = 0;
    const float* g_scan = nullptr;
    const int* g_scan_n = nullptr;
    std::string err;
    int* h_cnt = nullptr;                // pinned copy of the counters
    int* h_err = nullptr;                // pinned copy of the counters for lo_devmap_status_async / _poll
    hipEvent_t ev_err = nullptr;         //   recorded after that copy
    bool err_pending = false;
    size_t updates = 0;
};

#define DM_HIP(m, x)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) { (m)->err = std::string(#x) + ": " + hipGetErrorString(e_); return LO_ERR_HIP; } \
    } while (0)

template <class T>
static int dm_alloc(lo_devmap* m, T** p, size_t count, int fill_byte) {
    void* v = nullptr;
    DM_HIP(m, hipMalloc(&v, std::max<size_t>(count, 1) * sizeof(T)));
    m->bufs.push_back(v);
    DM_HIP(m, hipMemset(v, fill_byte, std::max<size_t>(count, 1) * sizeof(T)));
    *p = static_cast<T*>(v);
    return LO_OK;
}

static int dm_fill_int(lo_devmap* m, int* p, size_t count, int value) {
    std::vector<int> h(count, value);
    DM_HIP(m, hipMemcpy(p, h.data(), count * sizeof(int), hipMemcpyHostToDevice));
    return LO_OK;
}

static uint32_t log2_at_least(size_t v) { uint32_t l = 1; while ((size_t(1) << l) < v) ++l; return l; }

// the context's table sized for the map (and emptied when it was replaced since): the ICP reads what we patch
static int dm_bind_table(lo_devmap* m) {
    void* tabv = nullptr;
    uint32_t l = 0;
    uint64_t gen = 0;
    const int rc = ctx_reserve_table(m->ctx, size_t(4) * static_cast<size_t>(m->M.C1), &tabv, &l, &gen);
    Slot* tab = static_cast<Slot*>(tabv);
    if (rc != LO_OK) { m->err = "context table: " + std::string(lo_last_error(m->ctx)); return rc; }
    if (gen != m->tab_gen) {                             // a fresh (empty) table: refill it from L1
        m->M.tab = tab;
        m->M.tabl = l;
        m->tab_gen = gen;
        hipLaunchKernelGGL(k_dm_flag, dim3(1), dim3(64), 0, m->stream, m->M, static_cast<int>(R_TAB));
        hipLaunchKernelGGL(k_dm_rebuild_clear, dim3(1024), dim3(kPar), 0, m->stream, m->M);
        hipLaunchKernelGGL(k_dm_rebuild_fill, dim3(1024), dim3(kPar), 0, m->stream, m->M);
        DM_HIP(m, hipGetLastError());
    }
    return LO_OK;
}

extern "C" {

lo_devmap* lo_devmap_create(lo_ctx* ctx, float voxel_size, int hierarchy_factor, float planarity_threshold,
                            size_t max_l0, size_t max_points, int* err) {
    auto fail = [&](int rc, const char* msg, lo_devmap* m) -> lo_devmap* {
        std::fprintf(stderr, "lo_devmap_create: %s\n", m && !m->err.empty() ? m->err.c_str() : msg);
        if (m) lo_devmap_destroy(m);
        if (err) *err = rc;
        return nullptr;
    };
    if (!ctx || !(voxel_size > 0.0f) || (hierarchy_factor != 1 && hierarchy_factor != 3) || max_l0 < 16 ||
        max_l0 > (size_t(1) << 26) || max_points < 1 || max_points > (size_t(1) << 24))
        return fail(LO_ERR_ARG, "bad arguments (factor 1 or 3, 16 <= max_l0 <= 2^26, max_points <= 2^24)", nullptr);
    lo_config cfg;
    if (lo_get_config(ctx, &cfg) != LO_OK) return fail(LO_ERR_ARG, "bad context", nullptr);
    // a KDTree-mode context reads the map's L0 centroids through its grid (lo_devmap_sync_points); the surfel table
    // the map keeps is then unused by its ICP
    lo_devmap* m = new lo_devmap();
    m->ctx = ctx;
    m->device = lo_device(ctx);
    m->stream = static_cast<hipStream_t>(lo_stream(ctx));
    if (hipSetDevice(m->device) != hipSuccess) return fail(LO_ERR_HIP, "hipSetDevice", m);
    DM& M = m->M;
    M.C0 = static_cast<int>(max_l0);
    M.C1 = static_cast<int>(std::max<size_t>(max_l0 / 2, 16));
    M.NP = static_cast<int>(max_points);
    M.h0l = log2_at_least(2 * static_cast<size_t>(M.C0));
    M.h1l = log2_at_least(2 * static_cast<size_t>(M.C1));
    M.hpl = log2_at_least(2 * std::max<size_t>(M.NP, 16));
    M.voxel = voxel_size;
    M.l1scale = voxel_size * static_cast<float>(hierarchy_factor);
    M.thr = planarity_threshold;
    M.factor = hierarchy_factor;
    M.surfels = cfg.use_surfel_correspondence ? 1 : 0;
    const size_t C0 = M.C0, C1 = M.C1, NP = M.NP;
    const size_t H0 = size_t(1) << M.h0l, H1 = size_t(1) << M.h1l, HP = size_t(1) << M.hpl;
    const size_t HT = std::max(HP, H0);                  // the point hash doubles as ApplyTransform's key hash
    int rc = LO_OK;
#define A(p, n, b) if (rc == LO_OK) rc = dm_alloc(m, &(p), (n), (b))
    A(M.k0, C0, 0); A(M.c0, 3 * C0, 0); A(M.n0p, C0, 0);
    A(M.k1, C1, 0); A(M.kids, C1 * kKids, 0); A(M.nk, C1, 0); A(M.has, C1, 0); A(M.nrm, 3 * C1, 0); A(M.cen, 3 * C1, 0);
    A(M.plan, C1, 0); A(M.last, C1, 0);
    A(M.i0k, H0, 0xff); A(M.i0v, H0, 0); A(M.i1k, H1, 0xff); A(M.i1v, H1, 0);
    A(M.cnt, 16, 0);
    A(M.flag, C0, 0); A(M.blkcnt, kPruneBlocks, 0); A(M.bc, 3 * kChunk, 0); A(M.bo, 3 * kChunk, 0); A(M.D, C0, 0); A(M.emptied, C0, 0); A(M.ucnt, C1, 0);
    A(M.ulist, C1 * kKids, 0); A(M.E1, std::max(C1, NP), 0); A(M.hole0, C0, 0); A(M.hole1, C1, 0); A(M.simg, 4 * C0, 0);
    A(M.chg, C0, 0);
    A(M.tpk, HT, 0xff); A(M.tpfirst, HT, 0); A(M.tpcnt, HT, 0); A(M.tpfill, HT, 0); A(M.tppos, HP, 0); A(M.tpoff, HT, 0);
    A(M.ttk, HP, 0xff); A(M.ttfirst, HP, 0);
    A(M.tqk, HP, 0xff); A(M.tqfirst, HP, 0); A(M.tqcnt, HP, 0); A(M.tqfill, HP, 0); A(M.tqlp, HP, 0); A(M.tqoff, HP, 0);
    A(M.pslot, std::max(NP, C0), 0); A(M.tslot, NP, 0); A(M.rslot, NP, 0); A(M.pkey0, NP, 0); A(M.pkey1, NP, 0);
    A(M.newlist, std::max(NP, C0), 0); A(M.glist, std::max(NP, C0), 0); A(M.rlist, NP, 0);
    A(M.T, NP, 0); A(M.tlp, NP, 0); A(M.fail, NP, 0); A(M.F, std::max(NP, C1), 0); A(M.Foff, NP, 0);
    A(M.L0e, NP * kKids, 0);
    A(m->d_in, 3 * NP, 0);
    A(M.prm, 16, 0); A(M.prm_n, 4, 0);
    A(m->at_c, 3 * C0, 0); A(m->at_k, C0, 0); A(m->at_nk, C0, 0); A(m->at_nc, 3 * C0, 0); A(m->at_nn, C0, 0);
#undef A
    if (const char* e = std::getenv("LO_DM_STAMPS"); e && std::atoi(e) && rc == LO_OK) rc = dm_alloc(m, &M.st, 64, 0);
    if (rc == LO_OK) rc = dm_fill_int(m, M.tpfirst, HT, INT_MAX);
    if (rc == LO_OK) rc = dm_fill_int(m, M.ttfirst, HP, INT_MAX);
    if (rc == LO_OK) rc = dm_fill_int(m, M.tqfirst, HP, INT_MAX);
    if (rc == LO_OK && hipHostMalloc(&m->h_cnt, 16 * sizeof(int), hipHostMallocDefault) != hipSuccess) rc = LO_ERR_HIP;
    if (rc == LO_OK && hipHostMalloc(&m->h_err, 16 * sizeof(int), hipHostMallocDefault) != hipSuccess) rc = LO_ERR_HIP;
    if (rc == LO_OK && hipEventCreateWithFlags(&m->ev_err, hipEventDisableTiming) != hipSuccess) rc = LO_ERR_HIP;
    if (rc == LO_OK) rc = dm_bind_table(m);
    if (rc == LO_OK && hipStreamSynchronize(m->stream) != hipSuccess) rc = LO_ERR_HIP;
    if (rc != LO_OK) return fail(rc, "allocation", m);
    if (err) *err = LO_OK;
    return m;
}

void lo_devmap_destroy(lo_devmap* m) {
    if (!m) return;
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    if (m->M.st && m->updates) {                          // LO_DM_STAMPS=1: per-phase cycles per update
        unsigned long long h[64];
        if (hipMemcpy(h, m->M.st, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess) {
            std::fprintf(stderr, "lo_devmap phase cycles per update (%zu updates):", m->updates);
            for (int k = 0; k < 64; ++k) if (h[k]) std::fprintf(stderr, " %d:%llu", k, h[k] / m->updates);
            std::fprintf(stderr, "\n");
        }
    }
    if (m->gexec) (void)hipGraphExecDestroy(m->gexec);
    for (void* p : m->bufs) (void)hipFree(p);
    if (m->h_cnt) (void)hipHostFree(m->h_cnt);
    if (m->h_err) (void)hipHostFree(m->h_err);
    if (m->ev_err) (void)hipEventDestroy(m->ev_err);
    delete m;
}

const char* lo_devmap_last_error(const lo_devmap* m) { return m ? m->err.c_str() : "null map"; }

// One update = the parameter kernel + a captured graph of the twenty pipeline launches (kernel arguments fixed: the
// map's buffers, its point buffer, the device count; recaptured when the context's table moved).
static int dm_capture(lo_devmap* m, const int* d_scan_n, const float* d_scan) {
    DM& M = m->M;
    if (m->gexec) { (void)hipGraphExecDestroy(m->gexec); m->gexec = nullptr; }
    hipGraph_t g = nullptr;
    DM_HIP(m, hipStreamBeginCapture(m->stream, hipStreamCaptureModeThreadLocal));
    const int* dn = M.prm_n;
    const dim3 grid(std::max(1, std::min(1024, (M.NP + kPar - 1) / kPar)));
    const dim3 tgrid(std::max(1, std::min(1024, (M.NP + 63) / 64)));
    const dim3 chunks(kChunk), par(kPar);
    hipLaunchKernelGGL(k_dm_world, grid, par, 0, m->stream, M, d_scan, d_scan_n, m->d_in);
    hipLaunchKernelGGL(k_dm_prune_mark, dim3(kPruneBlocks), par, 0, m->stream, M, dn);
    hipLaunchKernelGGL(k_dm_prune_compact, dim3(kPruneBlocks), par, 0, m->stream, M, dn);
    hipLaunchKernelGGL(k_dm_unregister, dim3(1), dim3(kOrch), 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_keys, grid, par, 0, m->stream, M, m->d_in, 0, dn);
    hipLaunchKernelGGL(k_dm_a_count, chunks, par, 0, m->stream, M, 0, dn);
    hipLaunchKernelGGL(k_dm_scan3, dim3(1), dim3(kOrch), 0, m->stream, M, 1);
    hipLaunchKernelGGL(k_dm_a_rank, chunks, par, 0, m->stream, M, 0, dn);
    hipLaunchKernelGGL(k_dm_a_fill, grid, par, 0, m->stream, M, 0, dn);
    hipLaunchKernelGGL(k_dm_a_mean, grid, par, 0, m->stream, M, m->d_in, 0, dn);
    hipLaunchKernelGGL(k_dm_r_group, grid, par, 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_r_count, chunks, par, 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_scan3, dim3(1), dim3(kOrch), 0, m->stream, M, 2);
    hipLaunchKernelGGL(k_dm_r_rank, chunks, par, 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_r_fill, grid, par, 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_r_append, grid, par, 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_a_done, grid, par, 0, m->stream, M, 0, dn);
    hipLaunchKernelGGL(k_dm_touched, tgrid, dim3(64), 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_finish, dim3(1), dim3(kOrch), 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_table, grid, par, 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_table_check, dim3(1), dim3(64), 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_rebuild_clear, dim3(1024), par, 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_rebuild_fill, dim3(1024), par, 0, m->stream, M);
    const hipError_t le = hipGetLastError();
    const hipError_t ce = hipStreamEndCapture(m->stream, &g);
    if (le != hipSuccess || ce != hipSuccess) {
        if (g) (void)hipGraphDestroy(g);
        m->err = std::string("graph capture: ") + hipGetErrorString(le != hipSuccess ? le : ce);
        return LO_ERR_HIP;
    }
    const hipError_t ie = hipGraphInstantiate(&m->gexec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (ie != hipSuccess) { m->gexec = nullptr; m->err = std::string("graph instantiate: ") + hipGetErrorString(ie); return LO_ERR_HIP; }
    m->g_tab = M.tab;
    m->g_tabl = M.tabl;
    m->g_scan = d_scan;
    m->g_scan_n = d_scan_n;
    return LO_OK;
}

// The map launches on its context's stream, looked up on every call (lo_set_stream may have replaced it; the captured
// update graph is stream-independent).
static void dm_stream(lo_devmap* m) { m->stream = static_cast<hipStream_t>(lo_stream(m->ctx)); }

static int dm_update(lo_devmap* m, int n_host, bool from_scan, const float T[12], const double sensor[3],
                     double max_distance) {
    DM& M = m->M;
    int rc = dm_bind_table(m);
    if (rc != LO_OK) return rc;
    const float* d_scan = nullptr;
    const int* d_scan_n = nullptr;
    if (from_scan) {
        rc = ctx_filtered_device(m->ctx, &d_scan, &d_scan_n);
        if (rc != LO_OK) { m->err = lo_last_error(m->ctx); return rc; }
    } else {
        d_scan = m->g_scan;                               // unused by the graph in this mode: keep it
        d_scan_n = m->g_scan_n ? m->g_scan_n : M.prm_n;
    }
    if (!m->gexec || m->g_tab != M.tab || m->g_tabl != M.tabl || (from_scan && (m->g_scan != d_scan || m->g_scan_n != d_scan_n))) {
        rc = dm_capture(m, d_scan_n, d_scan);
        if (rc != LO_OK) return rc;
    }
    DmParams P{};
    P.v[0] = static_cast<float>(sensor[0]);
    P.v[1] = static_cast<float>(sensor[1]);
    P.v[2] = static_cast<float>(sensor[2]);
    P.v[3] = static_cast<float>(max_distance * max_distance);
    if (T) std::memcpy(P.v + 4, T, 12 * sizeof(float));
    P.n = n_host;
    P.from_scan = from_scan ? 1 : 0;
    ++m->updates;
    hipLaunchKernelGGL(k_dm_setprm, dim3(1), dim3(64), 0, m->stream, M, P);
    DM_HIP(m, hipGetLastError());
    DM_HIP(m, hipGraphLaunch(m->gexec, m->stream));
    return LO_OK;
}

int lo_devmap_update(lo_devmap* m, const float* world_xyz, size_t n, int on_device, const double sensor[3],
                     double max_distance, int is_keyframe) {
    if (!m || !sensor || (n > 0 && !world_xyz)) return LO_ERR_ARG;
    if (n == 0 || !is_keyframe) return LO_OK;           // UpdateVoxelMap returns before pruning (:135-142)
    if (n > static_cast<size_t>(m->M.NP)) { m->err = "more points than max_points"; return LO_ERR_CAPACITY; }
    DM_HIP(m, hipSetDevice(m->device));
    dm_stream(m);
    DM_HIP(m, hipMemcpyAsync(m->d_in, world_xyz, n * 3 * sizeof(float),
                             on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, m->stream));
    return dm_update(m, static_cast<int>(n), false, nullptr, sensor, max_distance);
}

int lo_devmap_update_from_scan(lo_devmap* m, const float T[12], double max_distance) {
    if (!m || !T) return LO_ERR_ARG;
    DM_HIP(m, hipSetDevice(m->device));
    dm_stream(m);
    const double sensor[3] = {T[3], T[7], T[11]};        // Vector3f -> Vector3d
    // an empty scan returns before the prune (UpdateVoxelMap :135-137): the kernels read the device count
    return dm_update(m, 0, true, T, sensor, max_distance);
}

int lo_devmap_apply_transform(lo_devmap* m, const float T[12]) {
    if (!m || !T) return LO_ERR_ARG;
    DM_HIP(m, hipSetDevice(m->device));
    dm_stream(m);
    int rc = dm_bind_table(m);
    if (rc != LO_OK) return rc;
    DM& M = m->M;
    DmPose P;
    std::memcpy(P.v, T, sizeof(P.v));
    const int G0 = (M.C0 + kPar - 1) / kPar;
    hipLaunchKernelGGL(k_dm_at_keys, dim3(G0), dim3(kPar), 0, m->stream, M, P, m->at_c, m->at_k);
    hipLaunchKernelGGL(k_dm_at_rebuild, dim3(1), dim3(kOrch), 0, m->stream, M, m->at_c, m->at_k, M.pslot, M.tpfirst,
                       M.tpcnt, M.tpoff, M.tpfill, M.glist, M.D, m->at_nk, m->at_nc, m->at_nn);
    hipLaunchKernelGGL(k_dm_flag, dim3(1), dim3(64), 0, m->stream, M, static_cast<int>(R_I0 | R_I1 | R_TAB));
    hipLaunchKernelGGL(k_dm_rebuild_clear, dim3(1024), dim3(kPar), 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_rebuild_fill, dim3(1024), dim3(kPar), 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_recompute, dim3((M.C1 + kPar - 1) / kPar), dim3(kPar), 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_flag, dim3(1), dim3(64), 0, m->stream, M, static_cast<int>(R_TAB));
    hipLaunchKernelGGL(k_dm_rebuild_clear, dim3(1024), dim3(kPar), 0, m->stream, M);
    hipLaunchKernelGGL(k_dm_rebuild_fill, dim3(1024), dim3(kPar), 0, m->stream, M);
    DM_HIP(m, hipGetLastError());
    return LO_OK;
}

int lo_devmap_status(lo_devmap* m) {
    if (!m) return LO_ERR_ARG;
    DM_HIP(m, hipSetDevice(m->device));
    dm_stream(m);
    DM_HIP(m, hipMemcpyAsync(m->h_cnt, m->M.cnt, 16 * sizeof(int), hipMemcpyDeviceToHost, m->stream));
    DM_HIP(m, hipStreamSynchronize(m->stream));
    if (m->h_cnt[C_ERR]) { m->err = "device map overflow / invalid key (error bits " + std::to_string(m->h_cnt[C_ERR]) + ")"; return LO_ERR_CAPACITY; }
    return LO_OK;
}

int lo_devmap_sync_points(lo_devmap* m) {
    if (!m) return LO_ERR_ARG;
    DM_HIP(m, hipSetDevice(m->device));
    dm_stream(m);
    const int rc = ctx_grid_from_device(m->ctx, m->M.c0, m->M.cnt + C_N0, static_cast<size_t>(m->M.C0));
    if (rc != LO_OK) m->err = std::string("sync_points: ") + lo_last_error(m->ctx);
    return rc;
}

int lo_devmap_status_async(lo_devmap* m) {
    if (!m) return LO_ERR_ARG;
    DM_HIP(m, hipSetDevice(m->device));
    dm_stream(m);
    DM_HIP(m, hipMemcpyAsync(m->h_err, m->M.cnt, 16 * sizeof(int), hipMemcpyDeviceToHost, m->stream));
    DM_HIP(m, hipEventRecord(m->ev_err, m->stream));
    m->err_pending = true;
    return LO_OK;
}

int lo_devmap_status_poll(lo_devmap* m) {
    if (!m) return LO_ERR_ARG;
    if (!m->err_pending) return LO_OK;
    const hipError_t q = hipEventQuery(m->ev_err);
    if (q == hipErrorNotReady) return LO_OK;             // still in flight: the next poll reads it
    DM_HIP(m, q);
    m->err_pending = false;
    if (m->h_err[C_ERR]) { m->err = "device map overflow / invalid key (error bits " + std::to_string(m->h_err[C_ERR]) + ")"; return LO_ERR_CAPACITY; }
    return LO_OK;
}

int lo_devmap_counts(lo_devmap* m, size_t out[4]) {
    if (!m || !out) return LO_ERR_ARG;
    DM_HIP(m, hipSetDevice(m->device));
    dm_stream(m);
    DM_HIP(m, hipMemcpyAsync(m->h_cnt, m->M.cnt, 16 * sizeof(int), hipMemcpyDeviceToHost, m->stream));
    DM_HIP(m, hipStreamSynchronize(m->stream));
    out[0] = static_cast<size_t>(m->h_cnt[C_N0]);
    out[1] = static_cast<size_t>(m->h_cnt[C_N1]);
    out[3] = static_cast<size_t>(m->h_cnt[C_ERR]);
    // surfels: counted from the L1 flags
    const int n1 = m->h_cnt[C_N1];
    std::vector<int> has(std::max(n1, 1));
    if (n1 > 0) DM_HIP(m, hipMemcpy(has.data(), m->M.has, n1 * sizeof(int), hipMemcpyDeviceToHost));
    size_t s = 0;
    for (int i = 0; i < n1; ++i) s += has[i] ? 1 : 0;
    out[2] = s;
    if (m->h_cnt[C_ERR]) { m->err = "device map overflow / invalid key (error bits " + std::to_string(m->h_cnt[C_ERR]) + ")"; return LO_ERR_CAPACITY; }
    return LO_OK;
}

size_t lo_devmap_get_l0(lo_devmap* m, int32_t* keys, float* xyz, int32_t* point_counts, size_t cap) {
    size_t c[4] = {0, 0, 0, 0};
    const int rc = lo_devmap_counts(m, c);
    if (rc != LO_OK && rc != LO_ERR_CAPACITY) return 0;
    const size_t n = std::min(c[0], cap);
    if (n == 0) return 0;
    std::vector<uint64_t> k(n);
    std::vector<float> x(3 * n);
    std::vector<int> pc(n);
    if (hipMemcpy(k.data(), m->M.k0, n * 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(x.data(), m->M.c0, n * 12, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(pc.data(), m->M.n0p, n * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return 0;
    for (size_t i = 0; i < n; ++i) {
        if (keys) for (int a = 0; a < 3; ++a) keys[3 * i + a] = static_cast<int32_t>((k[i] >> (21 * a)) & 0x1FFFFF) - (1 << 20);
        if (xyz) for (int a = 0; a < 3; ++a) xyz[3 * i + a] = x[3 * i + a];
        if (point_counts) point_counts[i] = pc[i];
    }
    return n;
}

size_t lo_devmap_get_l1(lo_devmap* m, int32_t* keys, uint8_t* has_surfel, float* normals, float* centroids,
                        float* planarity, int32_t* child_counts, int32_t* children, size_t cap) {
    size_t c[4] = {0, 0, 0, 0};
    const int rc = lo_devmap_counts(m, c);
    if (rc != LO_OK && rc != LO_ERR_CAPACITY) return 0;
    const size_t n = std::min(c[1], cap);
    if (n == 0) return 0;
    std::vector<uint64_t> k(n), kids(n * kKids);
    std::vector<int> nk(n), has(n);
    std::vector<float> nr(3 * n), ce(3 * n), pl(n);
    if (hipMemcpy(k.data(), m->M.k1, n * 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(kids.data(), m->M.kids, n * kKids * 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(nk.data(), m->M.nk, n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(has.data(), m->M.has, n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(nr.data(), m->M.nrm, n * 12, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(ce.data(), m->M.cen, n * 12, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(pl.data(), m->M.plan, n * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return 0;
    auto unp = [](uint64_t v, int a) { return static_cast<int32_t>((v >> (21 * a)) & 0x1FFFFF) - (1 << 20); };
    for (size_t i = 0; i < n; ++i) {
        if (keys) for (int a = 0; a < 3; ++a) keys[3 * i + a] = unp(k[i], a);
        if (has_surfel) has_surfel[i] = has[i] ? 1 : 0;
        for (int a = 0; a < 3; ++a) {
            if (normals) normals[3 * i + a] = nr[3 * i + a];
            if (centroids) centroids[3 * i + a] = ce[3 * i + a];
        }
        if (planarity) planarity[i] = pl[i];
        if (child_counts) child_counts[i] = nk[i];
        if (children)
            for (int q = 0; q < kKids; ++q)
                for (int a = 0; a < 3; ++a)
                    children[(i * kKids + q) * 3 + a] = q < nk[i] ? unp(kids[i * kKids + q], a) : 0;
    }
    return n;
}

}  // extern "C"
