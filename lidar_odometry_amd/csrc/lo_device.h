// lo_device.h — device-side data layout and numerics shared by the ICP kernels (gfx950 / CDNA4).
//
// HBM layout (one context):
//   scan points       AoS float3, 12 B/pt (Point3D as the reference stores it; coalesced dwordx3 loads)
//   surfel table      open-addressing hash, power-of-two capacity, load <= 0.5, linear probing;
//                     one 32-B slot = {u64 Morton key, float normal[3], float centroid[3]} so a probe that
//                     hits brings the payload in the same 32-B sector (no dependent second miss)
//   per point         int32 slot index of the accepted correspondence (-1 = none)
//   per 64 points     u64 validity ballot (rank -> point mapping for the PKO sampler)
//   per 256-pt block  int count, fp64 residual sum and M2 (iteration-0 scale), 28 fp64 normal-eq partials
//   DevState          pose, scale, alpha, n_corr, done flag, per-iteration logs (the GN loop state
//                     lives on the device; the host never syncs inside optimize)
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../../include/lo_icp.h"
#include "lo_kdorder.h"

namespace lo {

constexpr int kBlock = 256;          // threads per block for the per-point kernels (4 waves)
constexpr int kWave = 64;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr uint64_t kEmptyKey = ~0ull;
constexpr uint64_t kTombKey = ~0ull - 1;   // erased slot (lo_map_patch_surfels): never a packed key, never empty
constexpr int kNE = 28;              // 21 lower-triangular H + 6 g + cost
constexpr int kPkoBlock = 256;       // PKO workgroup: one GMM sample per thread (S <= 256)
constexpr int kPkoMaxWGs = 128;      // PKO workgroups per launch (each evaluates a slice of the alpha grid)
constexpr int kMaxBlocks = 16384;    // => max 4M points per scan
constexpr int kAccBlocks = 1024;     // k_accumulate grid cap (grid-stride beyond): bounds the k_solve partial sum
constexpr int kSolveThreads = 1024;  // k_solve: 36 x 28 threads sum the block partials, coalesced
constexpr int kFuseMaxBlocks = 64;   // <= this many accumulate blocks: the last one also solves (no k_solve launch)
constexpr int kMaxS = 256;
constexpr int kMaxK = 4;
constexpr int kMaxAlpha = 1000;
constexpr int kKnnGroup = 16;       // KDTree k_knn: lanes per query (one DPP row)
constexpr int kKnnAllMax = 8192;     // k_knn_all / k_inlier_all: points of a set searched whole from LDS (128 KB)
constexpr int kAllThreads = 1024;    // k_knn_all / k_pick_knn_all / k_inlier_all: 16 queries (a wave each) per workgroup
constexpr int kSpecBlocksPerWG = 16; // speculative normal equations: 256-point blocks per candidate workgroup
constexpr int kCandWords = 48;      // a candidate's solved GN step: pose[12] | cost | H[21] | g[6] | delta[6] | conv | pad
constexpr int kCandCost = 12, kCandH = 13, kCandG = 34, kCandD = 40, kCandConv = 46;
// reference-exact candidates (lo_pko_body.h acc_candidate_exact): the 43 terms of a chunk's points staged term-major
// in the PKO launch's dynamic LDS (4 consecutive rows of one term per ds_read_b128)
constexpr int kSpanStarts = 16, kSpanEnds = 256;            // KParams::span: plain per-block stores, no atomics
constexpr int kSpanWords = kSpanStarts + kSpanEnds;
constexpr int kXcRegions = 3;                              // 64-point regions per chunk (one per producer wave)
constexpr int kXcChunk = kXcRegions * kWave;              // 192 points
constexpr int kXcPad = 16;                                 // a chunk's staged rows padded to a multiple of 16
constexpr int kXcFactors = 14;                             // a point's factors (J, wJ, wr, r): every term is fa * fb
// floats per factor row: a chunk's rows + padding, and 212 = 20 mod 64 puts the 14 rows' 16-B reads on disjoint banks
constexpr int kXcStride = 212;
static_assert(kXcStride >= kXcChunk + kXcPad - 1, "a padded chunk fits a factor row");
constexpr int kXcBuf = kXcFactors * kXcStride;             // one chunk's factor rows
constexpr int kXcCntOff = 2 * kXcBuf;                      // [4][kXcRegions] valid rows per region (ints)
constexpr int kXcTotOff = kXcCntOff + 4 * kXcRegions;      // [43] the sums, then the candidate record
constexpr size_t kXcLdsBytes = (kXcTotOff + 43 + kCandWords) * sizeof(float);

struct __attribute__((aligned(32))) Slot {
    uint64_t key;
    float n[3];
    float c[3];
};
static_assert(sizeof(Slot) == 32, "slot must be one 32-B sector");

struct DevState {
    float pose[12];
    double scale;
    double alpha;
    int n_corr;
    int iter;
    int done;
    int status;
    unsigned int acc_arrive;        // k_accumulate last-block-done counter (reset by the last block)
    unsigned int kd_unres_n;        // KDTree path: queries the grid search could not certify (k_knn_brute)
    unsigned int inliers;           // loop closure: points whose nearest matched-map point is < 1 m (k_inlier)
    unsigned int kd_tie;            // KDTree grid without its kd visit order: a query met a deciding distance tie
    double H_out[36];
    double g_out[6];
    double cost_out;
    double gmm_out[3 * kMaxK];
    unsigned long long dbg[24];     // diagnostic builds: phase timestamps / counters; product: [5] / [8] long-sum walk
                                    // statistics, [23] the last one-workgroup exact scale's sort width (points)
    unsigned long long em_stat[3];  // with stage timing: EM s_memtime cycles, EM iterations, fits (lead workgroup)
    lo_iter_log logs[LO_MAX_ITERS];
};

struct KParams;
struct KParams {
    // scan
    const float* pts;
    int n;                            // points (upper bound when n_dev is set)
    const int* n_dev;                 // device-side point count (device voxel filter output), or null
    int nb;
    int nb_acc;                       // k_accumulate blocks = min(nb, kAccBlocks)
    int init;                         // k_correspond: first launch of a scan resets DevState (pose = T0)
    float T0[12];
    const float* T0p;                 // batched launches: the job's initial pose in device memory (else T0)
    // KDTree correspondence path (use_surfel_correspondence = 0; lo_kdtree.hip)
    const float4* kd_pts;             // L0 centroids sorted by grid cell: x, y, z, original index (int bits)
    const uint32_t* kd_start;         // cell -> first point (dense grid, ncell + 1 entries)
    const uint32_t* kd_vpos;          // reference kd-tree visit order (lo_kdorder.h): vAcc_ position per index
    const KdNode* kd_nodes;    //   and its nodes, for equal-distance tie-breaks
    int kd_m;                         // map points
    int kd_org[3], kd_dim[3];         // grid origin (cell coords) and extent
    float kd_h;                       // grid cell edge
    int kd_all;                       // kd_pts is a small set in index order searched whole from LDS (k_knn_all)
    int32_t* kd_nbr;                  // per point: 5 neighbour positions into kd_pts (-1: fewer than 5)
    int32_t* kd_unres;                // queries left to the brute-force pass
    double* kd_res;                   // per point fp64 point-to-plane distance (the reference's residual)
    Slot* kd_plane;                   // per point plane: normal / centroid rounded to fp32 (.cast<float>())
    // loop-closure ICP (optimize_loop, IterativeClosestPointOptimizer.cpp:40-251): no distance gate, and the
    // target is neighbour 0 taken to the matched keyframe's local frame (Tlw) and back to the world (Tm)
    int loop;
    float Tm[12];                     // matched keyframe pose, row-major 3x4
    float Tlw[12];                    // its inverse (T_lw_last, :509)
    // map
    const Slot* tab;
    uint32_t log2cap;
    float l1scale;
    // ICP config
    int max_iters;
    double tol_t, tol_r, maxd;
    int min_corr;
    int robust;
    double robust_delta;
    int cauchy_loss;
    int use_pko;
    int alpha_given;          // 1: take the Huber delta from DevState::alpha (normal-equation entry point)
    // PKO config + tables
    int S, K, NA, pko_kernel;           // pko_kernel: LO_PKO_*
    double min_scale, trunc;
    const double* alphas;
    const double* Z;
    const int32_t* small_off;
    const int32_t* small_perm;
    const int32_t* base;
    const int32_t* ev_off;
    const int32_t* ev_steps;
    const int32_t* km_draws;
    // work buffers
    int32_t* slot;
    uint64_t* wmask;
    int32_t* blk_cnt;
    double* blk_sum;
    double* blk_m2;
    double* blk_part;
    double* acc_part;         // speculative normal equations: [NA + 1 candidates][kFuseMaxBlocks][kNE] partials
    float* cand_rec;          // nullable: each candidate's solved GN step [NA + 1][kCandWords] (pre-solved in the PKO
                              //   launch while the EM runs; k_pick_correspond / k_pick select one)
    unsigned* cand_cnt;       //   per-candidate arrivals of its W workgroups (the last one solves and re-zeroes it)
    double* js;               // [NA+1] JS divergence per alpha (k_pko -> argmin in the consumers)
    double* res_dbg;          // nullable: per-point residual (parity entry point)
    unsigned long long* span; // nullable (timing, kSpanWords): start stamps of blocks 0-15, end stamps of the last 256
                              //   blocks of this correspondence launch, s_memrealtime (100 MHz); preset ~0 / 0
    double* res_out;          // nullable: per-point fp64 residual of the accepted correspondences (k_correspond /
                              //   k_solve_correspond), read back by the PKO sample instead of recomputing it
    float* ex_terms;          // reference-exact mode (lo_exact.hip): per point the 43 fp32 normal-equation terms
    int ex_ld;                //   0: row-major [point][43]; > 0: term-major [43][ex_ld] (large scans, launch_mw_sums)
    float* ex_tot;            //   term-major path: the 43 sequential sums
    int scale_given;          // 1: the iteration-0 scale is already in DevState (k_exact_scale), the PKO reads it
    uint64_t* presort;        // nullable (iteration 0, reference-exact mode): each correspondence block writes its 256
                              //   residual keys sorted (lo_blocksort.h) for k_exact_scale_m's merge
    int exact_cand;           // 1: the PKO launch's candidates form the reference's sequential fp32 sums and solve
                              //   (reference-exact mode, acc_candidate_exact; one workgroup per candidate)
    const double* direct_res; // nullable: PKO on given residuals (parity entry point)
    unsigned long long* em_stat;  // nullable (stage timing on): DevState::em_stat, the lead PKO workgroup's EM timing
    DevState* st;
    uint32_t* fin;            // nullable (scan pipeline, lo_set_pipeline): the context's "last final scan" word
                              //   (fin[1] main part done, fin[2] signal_main's block count, fin[3] pipeline broken)
    uint32_t seq;             //   and this scan's sequence number, published there once its result is final
    int hold;                 // 1: the main part's last pick (signal_main: fin[1] = seq once its correspondences are out;
                              //   fin[2] counts its blocks in)
    int tail;                 // 1: a tail-stream launch -- it leaves once scan seq is final (fin_reached; the DevState may
                              //   then already be the next scan's) and reads the caller's points only after that test
};

// Scan pipeline: the thread that wrote a scan's final DevState (pose, logs, status) writes it back to memory (agent
// release: every XCD and the copy engines read the fresh bytes) and then publishes the scan's sequence number with
// an sc1 store; k_wait_final (and k_wait_seq) poll that word (MI355X_MICROARCH.md "inter-workgroup
// visibility": release, then the explicit vmcnt wait, then the relaxed agent-scope flag store).
// Scan pipeline: poll a flag word until it reaches seq (one lane, sc1 loads: fresh across XCDs; the word is the only
// thing read), bounded by `bound` ticks of the 100 MHz constant clock -- false on timeout, so no wait can hang a queue.
// A wait also gives up at once when the pipeline is broken (fin[3] != 0: an earlier wait timed out).
__device__ __forceinline__ bool wait_word(const uint32_t* w, uint32_t seq, const uint32_t* broken, unsigned long long bound) {
    const unsigned long long t0 = wall_clock64();
    while (static_cast<int32_t>(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - seq) < 0) {
        if (__hip_atomic_load(broken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return false;
        if (wall_clock64() - t0 > bound) return false;
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}
// ... until either of two words reaches seq
__device__ __forceinline__ bool wait_word2(const uint32_t* a, const uint32_t* b, uint32_t seq, const uint32_t* broken,
                                           unsigned long long bound) {
    const unsigned long long t0 = wall_clock64();
    while (static_cast<int32_t>(__hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - seq) < 0 &&
           static_cast<int32_t>(__hip_atomic_load(b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - seq) < 0) {
        if (__hip_atomic_load(broken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return false;
        if (wall_clock64() - t0 > bound) return false;
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}

// A tail-stream launch's own early-exit test (sc1 load: fresh across XCDs; the scans become final in order).
__device__ __forceinline__ bool fin_reached(const KParams& P) {
    return static_cast<int32_t>(__hip_atomic_load(P.fin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - P.seq) >= 0;
}
// ... and the sticky "pipeline broken" word: once a wait has timed out, the two streams are no longer ordered against
// each other, so no tail launch may touch the context's buffers (they may already belong to a later scan).
__device__ __forceinline__ bool pipe_broken(const KParams& P) {
    return __hip_atomic_load(P.fin + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}
__device__ __forceinline__ bool tail_gone(const KParams& P) { return P.tail && (fin_reached(P) || pipe_broken(P)); }
__device__ __forceinline__ void publish_final(const KParams& P) {
    if (!P.fin) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(P.fin, P.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The per-iteration buffers a PKO pass works on (own_bufs: the context's own), passed beside the kernel-argument
// KParams.
struct ScanBufs {
    int32_t* slot;
    uint64_t* wmask;
    int32_t* blk_cnt;
    double* js;
    DevState* st;
    const float* pose_in;             // the iteration's pose (nullable: st->pose)
    const double* res;                // the correspondences' residuals (nullable: recomputed from slot + pose)
};
__device__ __forceinline__ ScanBufs own_bufs(const KParams& P) {
    return ScanBufs{P.slot, P.wmask, P.blk_cnt, P.js, P.st, nullptr, P.res_out};
}

// ---------------------------------------------------------------------------------------------------
// Memory policy of the buffers one workgroup hands to another INSIDE a launch (a speculative candidate's W > 1
// workgroups, whose last arrival solves: lo_pko_body.h acc_candidate).  Mem<false>: plain loads / stores (the
// hand-off is a kernel boundary).  Mem<true>: agent-scope
// relaxed atomic loads / stores on the global address space -- `global_load/store ... sc1`: stores write through
// the XCD's L2, loads bypass the CU's L1 -- so a consumer that saw the producer's counter after the producer drained
// its stores (s_waitcnt vmcnt(0)) reads the fresh bytes on any XCD without release / acquire fences
// (MI355X_MICROARCH.md "inter-workgroup visibility", the one-lane-signals / sc1-poll row).  Every load of a handed-off
// word in such a launch must go through Mem<true> (never the scalar path).
// ---------------------------------------------------------------------------------------------------
typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef __attribute__((address_space(1))) unsigned long long g_u64;

// A load through the global address space (global_load, counted by vmcnt only).  Pointers read from a KParams in
// memory (the batch kernels) or passed through helpers are generic, and a generic (flat) load is counted by lgkmcnt as
// well: then every wait for an LDS write before a barrier also waits for the loads in flight -- prefetches included.
template <typename T> __device__ __forceinline__ T gld(const T* p) {
    return *(const __attribute__((address_space(1))) T*)(p);
}

// a whole 32-B slot as two 16-B global loads (a builtin vector type: a class type's copy would bind a generic
// reference and load through flat again)
__device__ __forceinline__ Slot gld_slot(const Slot* p) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f a = gld(reinterpret_cast<const v4f*>(p)), b = gld(reinterpret_cast<const v4f*>(p) + 1);
    Slot s;
    s.key = static_cast<uint64_t>(__float_as_uint(a.x)) | (static_cast<uint64_t>(__float_as_uint(a.y)) << 32);
    s.n[0] = a.z; s.n[1] = a.w; s.n[2] = b.x;
    s.c[0] = b.y; s.c[1] = b.z; s.c[2] = b.w;
    return s;
}

template <bool SC1> struct Mem;
template <> struct Mem<false> {
    template <typename T> __device__ static __forceinline__ T ld(const T* p) { return *p; }
    template <typename T> __device__ static __forceinline__ void st(T* p, T v) { *p = v; }
};
template <> struct Mem<true> {
    template <typename T> __device__ static __forceinline__ T ld(const T* p) {
        static_assert(sizeof(T) == 4 || sizeof(T) == 8, "4- or 8-byte words");
        if constexpr (sizeof(T) == 4) {
            const uint32_t u = __hip_atomic_load((g_u32*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return __builtin_bit_cast(T, u);
        } else {
            const unsigned long long u = __hip_atomic_load((g_u64*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return __builtin_bit_cast(T, u);
        }
    }
    template <typename T> __device__ static __forceinline__ void st(T* p, T v) {
        static_assert(sizeof(T) == 4 || sizeof(T) == 8, "4- or 8-byte words");
        if constexpr (sizeof(T) == 4)
            __hip_atomic_store((g_u32*)(p), __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            __hip_atomic_store((g_u64*)(p), __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
};

// ---------------------------------------------------------------------------------------------------
// Bit-faithful scalar numerics (compiled with -ffp-contract=off; see DESIGN.md "fp order")
// ---------------------------------------------------------------------------------------------------

// transform_point_cloud: Matrix4f * Vector4f(x,y,z,1) (PointCloudUtils.cpp:119-121), Eigen packet order
__device__ __forceinline__ void transform_pt(const float* T, float x, float y, float z, float& ox, float& oy, float& oz) {
    float a;
    a = T[0] * x; a = T[1] * y + a; a = T[2] * z + a; a = T[3] * 1.0f + a; ox = a;
    a = T[4] * x; a = T[5] * y + a; a = T[6] * z + a; a = T[7] * 1.0f + a; oy = a;
    a = T[8] * x; a = T[9] * y + a; a = T[10] * z + a; a = T[11] * 1.0f + a; oz = a;
}

// 3-term fp32 dot (Eigen redux_novec_unroller order)
__device__ __forceinline__ float dot3f(float a0, float a1, float a2, float b0, float b1, float b2) {
    float e0 = a0 * b0, e1 = a1 * b1, e2 = a2 * b2;
    return e0 + (e1 + e2);
}

__device__ __forceinline__ bool key_in_range(int v) { return v >= -(1 << 20) && v < (1 << 20); }

__device__ __forceinline__ uint32_t hash_slot(uint64_t key, uint32_t log2cap) {
    return static_cast<uint32_t>((key * 0x9E3779B97F4A7C15ull) >> (64 - log2cap));
}

// Table key of an L1 voxel: the three 21-bit fields (key + 2^20) packed side by side.  The reference hashes
// VoxelKey with a Morton interleave (VoxelKeyHash, VoxelMap.h:166-183) but compares full keys; any injective
// packing gives the same hit / miss set, and packing costs 4 ALU ops against ~60 for the interleave.
__device__ __forceinline__ uint64_t pack_key(int kx, int ky, int kz) {
    return static_cast<uint64_t>(static_cast<uint32_t>(kx + (1 << 20))) |
           (static_cast<uint64_t>(static_cast<uint32_t>(ky + (1 << 20))) << 21) |
           (static_cast<uint64_t>(static_cast<uint32_t>(kz + (1 << 20))) << 42);
}

// Surfel lookup (VoxelMap::GetSurfelAtPoint :368-386): PointToVoxelKey(p, 1) (:50-58: fp32 division by
// voxel*factor, floor), then linear probing on the 8-B keys.  Returns the slot index or -1; the caller loads
// the 32-B slot (same sector, an L1/L2 hit).
__device__ __forceinline__ int lookup_surfel(const Slot* __restrict__ tab, uint32_t log2cap, float l1scale,
                                             float wx, float wy, float wz) {
    if (!(isfinite(wx) && isfinite(wy) && isfinite(wz))) return -1;
    const float fx = floorf(wx / l1scale), fy = floorf(wy / l1scale), fz = floorf(wz / l1scale);
    if (!(fx >= -1048576.0f && fx < 1048576.0f && fy >= -1048576.0f && fy < 1048576.0f &&
          fz >= -1048576.0f && fz < 1048576.0f)) return -1;
    const uint64_t key = pack_key(static_cast<int>(fx), static_cast<int>(fy), static_cast<int>(fz));
    const uint32_t mask = (1u << log2cap) - 1u;
    uint32_t h = hash_slot(key, log2cap);
    for (uint32_t p = 0; p <= mask; ++p) {
        const uint64_t k = tab[h].key;
        if (k == key) return static_cast<int>(h);
        if (k == kEmptyKey) return -1;
        h = (h + 1u) & mask;
    }
    return -1;
}

// fp64 point-to-plane residual |n.(p_w - c)| (IterativeClosestPointOptimizer.cpp:623-628);
// Vector3d dot in Eigen's Packet2d order: (e0 + e1) + e2
__device__ __forceinline__ double residual_f64(const Slot& s, float wx, float wy, float wz) {
    const double d0 = static_cast<double>(wx) - static_cast<double>(s.c[0]);
    const double d1 = static_cast<double>(wy) - static_cast<double>(s.c[1]);
    const double d2 = static_cast<double>(wz) - static_cast<double>(s.c[2]);
    const double e0 = static_cast<double>(s.n[0]) * d0;
    const double e1 = static_cast<double>(s.n[1]) * d1;
    const double e2 = static_cast<double>(s.n[2]) * d2;
    return fabs((e0 + e1) + e2);
}

// ---------------------------------------------------------------------------------------------------
// Wave-wide sums with DPP (quad_perm, row_half_mirror, row_mirror, row_bcast:15/31): 6 VALU steps and
// no LDS round trip (a __shfl_xor is a ds_bpermute through the LDS crossbar).  All 64 lanes must be
// active.  The total ends in lane 63 and is broadcast with v_readlane.
// ---------------------------------------------------------------------------------------------------
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int dpp32(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xf, false);
}
// full row mask: v_mov_b32_dpp without an "old" operand (no zeroing move in front of every DPP step)
template <int CTRL>
__device__ __forceinline__ int dpp32m(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false);
}
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp64(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const int lo = ROW_MASK == 0xf ? dpp32m<CTRL>(static_cast<int>(static_cast<uint32_t>(u)))
                                   : dpp32<CTRL, ROW_MASK>(static_cast<int>(static_cast<uint32_t>(u)));
    const int hi = ROW_MASK == 0xf ? dpp32m<CTRL>(static_cast<int>(static_cast<uint32_t>(u >> 32)))
                                   : dpp32<CTRL, ROW_MASK>(static_cast<int>(static_cast<uint32_t>(u >> 32)));
    return __builtin_bit_cast(double, (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo));
}

__device__ __forceinline__ double wave_total(double v) {
    v += dpp64<0xB1, 0xf>(v);    // quad_perm [1,0,3,2]
    v += dpp64<0x4E, 0xf>(v);    // quad_perm [2,3,0,1]
    v += dpp64<0x141, 0xf>(v);   // row_half_mirror
    v += dpp64<0x140, 0xf>(v);   // row_mirror        -> every lane holds its 16-lane row sum
    v += dpp64<0x142, 0xa>(v);   // row_bcast:15 into rows 1, 3
    v += dpp64<0x143, 0xc>(v);   // row_bcast:31 into rows 2, 3 -> lane 63 holds the total
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(u)), 63));
    const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(u >> 32)), 63));
    return __builtin_bit_cast(double, (static_cast<uint64_t>(hi) << 32) | lo);
}

__device__ __forceinline__ float wave_total(float v) {
#define LO_DPPF(CTRL, RM) __builtin_bit_cast(float, (RM) == 0xf ? dpp32m<CTRL>(__builtin_bit_cast(int, v)) : dpp32<CTRL, RM>(__builtin_bit_cast(int, v)))
    v += LO_DPPF(0xB1, 0xf);
    v += LO_DPPF(0x4E, 0xf);
    v += LO_DPPF(0x141, 0xf);
    v += LO_DPPF(0x140, 0xf);
    v += LO_DPPF(0x142, 0xa);
    v += LO_DPPF(0x143, 0xc);
#undef LO_DPPF
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

// Totals of NV <= 32 fp32 values over the 64 lanes of a wave, written to dst[0..NV) -- the normal-equation partials
// of one wave (28 values) in ~70 VALU ops instead of 28 DPP reductions (~200).  A butterfly that halves the values
// per lane while it halves the lane group: v_permlane32_swap (lanes l, l + 32), v_permlane16_swap (rows 0-1, 2-3),
// DPP row_ror:8 (l ^ 8), row_half_mirror (p <-> 7 - p in each 8-lane half row), quad_perm 2301 (l ^ 2) and 1032
// (l ^ 1); lane l ends with the total of value 16 b5 + 8 b4 + 4 b3 + 2 b2 + b1 (b = bits of l), which the even
// lane stores.  A fixed pairing tree (deterministic; not the per-value DPP tree of wave_total).
__device__ __forceinline__ void pl32_swapf(float& a, float& b) {   // a <- [a_lo | b_lo], b <- [a_hi | b_hi]
    const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b),
                                                    false, false);
    a = __builtin_bit_cast(float, static_cast<unsigned>(r[0]));
    b = __builtin_bit_cast(float, static_cast<unsigned>(r[1]));
}
__device__ __forceinline__ void pl16_swapf(float& a, float& b) {   // a <- rows [a0 b0 a2 b2], b <- [a1 b1 a3 b3]
    const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b),
                                                    false, false);
    a = __builtin_bit_cast(float, static_cast<unsigned>(r[0]));
    b = __builtin_bit_cast(float, static_cast<unsigned>(r[1]));
}
template <int CTRL>
__device__ __forceinline__ float dppf(float v) { return __builtin_bit_cast(float, dpp32m<CTRL>(__builtin_bit_cast(int, v))); }

template <int NV>
__device__ __forceinline__ void wave_totals_f32(const float (&v)[NV], float* dst) {
    static_assert(NV >= 1 && NV <= 32, "butterfly handles up to 32 values");
    const int lane = threadIdx.x & 63;
    float u[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) u[q] = q < NV ? v[q] : 0.0f;
#pragma unroll
    for (int q = 0; q < 16; ++q) { pl32_swapf(u[q], u[q + 16]); u[q] += u[q + 16]; }
#pragma unroll
    for (int q = 0; q < 8; ++q) { pl16_swapf(u[q], u[q + 8]); u[q] += u[q + 8]; }
    const bool b3 = (lane & 8) != 0, b2 = (lane & 4) != 0, b1 = (lane & 2) != 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float t = b3 ? u[q + 4] : u[q], o = b3 ? u[q] : u[q + 4];
        u[q] = t + dppf<0x128>(o);                        // row_ror:8
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const float t = b2 ? u[q + 2] : u[q], o = b2 ? u[q] : u[q + 2];
        u[q] = t + dppf<0x141>(o);                        // row_half_mirror
    }
    float t = b1 ? u[1] : u[0];
    const float o = b1 ? u[0] : u[1];
    t += dppf<0x4E>(o);                                   // quad_perm [2,3,0,1]
    t += dppf<0xB1>(t);                                   // quad_perm [1,0,3,2]
    const int idx = ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 + ((lane >> 2) & 1) * 2 +
                    ((lane >> 1) & 1);
    if ((lane & 1) == 0 && idx < NV) dst[idx] = t;
}

// fp64 reciprocal / reciprocal square root: v_rcp_f64 / v_rsq_f64 + two Newton steps (~1 ulp; ~5 VALU
// instead of the ~10 of a correctly rounded v_div_scale/v_div_fmas/v_div_fixup division).  A zero divisor
// gives NaN (0*inf in the Newton step) where IEEE division gives inf; every such use in the PKO feeds a
// quantity the reference also turns into NaN (0/0 responsibilities, empty components).
__device__ __forceinline__ double rcp64(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}
// One Newton step (~2^-48 relative): the EM's per-iteration reciprocals, whose results only need the GMM's
// tolerance (the fitted parameters are already tree sums, ~1e-9 from the reference), one dependent FMA pair shorter.
__device__ __forceinline__ double rcp64_1n(double x) {
    const double r = __builtin_amdgcn_rcp(x);
    return fma(r, fma(-x, r, 1.0), r);
}
__device__ __forceinline__ double rsq64_1n(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    return fma(0.5 * y, fma(-x * y, y, 1.0), y);
}
__device__ __forceinline__ double rsq64(double x) {
    double y = __builtin_amdgcn_rsq(x);
    double e = fma(-x * y, y, 1.0);
    y = fma(0.5 * y, e, y);
    e = fma(-x * y, y, 1.0);
    return fma(0.5 * y, e, y);
}

// std::max(a, b) for doubles (returns a when the comparison is false, so a NaN first argument survives)
__device__ __forceinline__ double std_max(double a, double b) { return (a < b) ? b : a; }

// calculate_pko_scale_factor's selection (AdaptiveMEstimator.cpp:256-275): the index of the FIRST alpha with
// the strictly smallest JS cost, 0 (min_scale_factor) if none is below DBL_MAX.  Every wave computes it
// redundantly from P.js (lexicographic (cost, index) minimum == first strict minimum).
__device__ __forceinline__ int pko_select_index(const KParams& P, const double* js) {
    const int lane = threadIdx.x & 63;
    double bv = 1.7976931348623157e308;
    int bi = 0x7fffffff;
    for (int i = 1 + lane; i <= P.NA; i += 64) {
        const double v = js[i];
        if (v < bv) { bv = v; bi = i; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov < bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    return (bv < 1.7976931348623157e308) ? bi : 0;
}
__device__ __forceinline__ int pko_select_index(const KParams& P) { return pko_select_index(P, P.js); }
__device__ __forceinline__ double pko_select_alpha(const KParams& P) {
    const int bi = pko_select_index(P);
    return bi > 0 ? P.alphas[bi] : P.min_scale;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Points of this scan: the host count, or the device voxel filter's count (lo_vfilter.hip) when the scan was
// filtered on the device -- grids are then sized for the upper bound and lanes past the count idle.
__device__ __forceinline__ int scan_n(const KParams& P) { return P.n_dev ? *P.n_dev : P.n; }

// ---------------------------------------------------------------------------------------------------
// Correspondence-kernel helpers shared by the surfel (k_correspond) and KDTree (lo_kdtree.hip) paths.
// ---------------------------------------------------------------------------------------------------
// Pose of the current GN iteration.  With init (first launch of a scan) it is the initial pose (kernel argument
// T0, or T0p in device memory for batched launches) and block 0 writes the fresh GN state that the later kernels
// of the scan read (k_init folded in).
__device__ __forceinline__ void scan_pose(const KParams& P, int init, int blk, float (&T)[12]) {
    DevState* st = P.st;
    if (init) {
#pragma unroll
        for (int k = 0; k < 12; ++k) T[k] = P.T0p ? P.T0p[k] : P.T0[k];
    } else {
#pragma unroll
        for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
    }
    if (init && blk == 0 && threadIdx.x < 12) {
        st->pose[threadIdx.x] = P.T0p ? P.T0p[threadIdx.x] : P.T0[threadIdx.x];
        if (threadIdx.x == 0) {
            st->scale = 1.0;
            st->alpha = P.robust_delta;
            st->n_corr = 0;
            st->iter = 0;
            st->done = 0;
            st->status = LO_OK;
            st->acc_arrive = 0;
            st->inliers = 0;
            st->kd_tie = 0;
            // kd_unres_n is NOT reset here: other blocks of the same k_knn launch may already be appending
            // (k_plane zeroes it after every use; k_init / lo_create start it at 0)
        }
    }
}

// Where a correspondence pass writes: per point the accepted slot and fp64 residual, per wave the validity ballot, per
// block the accepted count and (iteration 0) the residual sum / M2: the context's own buffers (corr_out(P)) or
// another set.
struct CorrOut {
    int32_t* slot;
    double* res;                      // nullable
    uint64_t* wmask;
    int32_t* blk_cnt;
    double* blk_sum;                  // with_stats only
    double* blk_m2;
};
__device__ __forceinline__ CorrOut corr_out(const KParams& P) {
    return CorrOut{P.slot, P.res_out, P.wmask, P.blk_cnt, P.blk_sum, P.blk_m2};
}

// Per-wave validity ballots, per-block accepted count and (iteration 0, with_stats) the per-block
// (count, sum, M2) of the accepted fp64 residuals for the stable merge of the residual variance.
__device__ __forceinline__ void corr_epilogue(const CorrOut& O, bool valid, double r, int with_stats, int vb) {
    __shared__ double s_red[kWavesPerBlock];
    __shared__ int s_cnt[kWavesPerBlock];
    __shared__ double s_mean;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t m = __ballot(valid);
    if (lane == 0) {
        O.wmask[vb * kWavesPerBlock + wid] = m;
        s_cnt[wid] = __popcll(m);
    }
    if (!with_stats) {
        __syncthreads();
        if (tid == 0) {
            int c = 0;
            for (int w = 0; w < kWavesPerBlock; ++w) c += s_cnt[w];
            O.blk_cnt[vb] = c;
        }
        return;
    }
    double v = wave_total(valid ? r : 0.0);
    if (lane == 0) s_red[wid] = v;
    __syncthreads();
    if (tid == 0) {
        int c = 0;
        double sum = 0.0;
        for (int w = 0; w < kWavesPerBlock; ++w) { c += s_cnt[w]; sum += s_red[w]; }
        O.blk_cnt[vb] = c;
        O.blk_sum[vb] = sum;
        s_mean = c > 0 ? sum / c : 0.0;
    }
    __syncthreads();
    const double mb = s_mean;
    const double d = valid ? (r - mb) : 0.0;
    v = wave_total(d * d);
    __syncthreads();
    if (lane == 0) s_red[wid] = v;
    __syncthreads();
    if (tid == 0) {
        double m2 = 0.0;
        for (int w = 0; w < kWavesPerBlock; ++w) m2 += s_red[w];
        O.blk_m2[vb] = m2;
    }
}
__device__ __forceinline__ void corr_epilogue(const KParams& P, bool valid, double r, int with_stats, int vb) {
    corr_epilogue(corr_out(P), valid, r, with_stats, vb);
}

// find_correspondences' per-point step (IterativeClosestPointOptimizer.cpp:606-641) for point i at pose T, then the
// block's ballots / count / (iteration 0) residual stats.
// Returns the point's sort key for the exact iteration-0 scale (lo_blocksort.h): the accepted residual's bits, else
// +inf's.
__device__ __forceinline__ uint64_t correspond_tail(const KParams& P, const CorrOut& O, const float (&T)[12], float px,
                                                    float py, float pz, int i, int n, int with_stats, int blk) {
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
        // streaming stores: read back only by the next kernels (PKO sample, accumulate), not by this launch
        __builtin_nontemporal_store(slot, &O.slot[i]);
        if (P.res_dbg) P.res_dbg[i] = slot >= 0 ? r : 0.0;
        if (O.res) __builtin_nontemporal_store(r, &O.res[i]);
    }
    corr_epilogue(O, slot >= 0, r, with_stats, blk);
    return slot >= 0 ? static_cast<uint64_t>(__double_as_longlong(r)) : 0x7FF0000000000000ull;
}
__device__ __forceinline__ uint64_t correspond_tail(const KParams& P, const float (&T)[12], float px, float py, float pz,
                                                    int i, int n, int with_stats, int blk) {
    return correspond_tail(P, corr_out(P), T, px, py, pz, i, n, with_stats, blk);
}

// ---------------------------------------------------------------------------------------------------
// One correspondence's weighted normal-equation terms added to acc (:345-410): residual, J, Huber weight,
// fp32 products fl(fl(w J_i) J_j) as the reference forms them.
// acc_terms: the terms of one correspondence from its loaded point / surfel and fp64 residual r.
__device__ __forceinline__ void acc_terms(const KParams& P, const float (&T)[12], double scale, float dl, double r,
                                          float px, float py, float pz, const Slot& sl, float (&acc)[kNE]) {
    const float nres = static_cast<float>(r / std_max(scale, 1e-6));          // :374
    // p_world = R p + t (Matrix3f * Vector3f, :368), residual n.(p_w - q) in fp32 (:371)
    const float qx = dot3f(T[0], T[1], T[2], px, py, pz) + T[3];
    const float qy = dot3f(T[4], T[5], T[6], px, py, pz) + T[7];
    const float qz = dot3f(T[8], T[9], T[10], px, py, pz) + T[11];
    const float n0 = sl.n[0], n1 = sl.n[1], n2 = sl.n[2];
    const float res = dot3f(n0, n1, n2, qx - sl.c[0], qy - sl.c[1], qz - sl.c[2]);
    // J = [n^T R, -n^T R [p]x] (:376-386)
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
    if (P.robust) {                                                             // :389-404
        const float an = fabsf(nres);
        if (P.cauchy_loss) { const float ratio = an / dl; w = 1.0f / (1.0f + ratio * ratio); }
        else if (an > dl) w = dl / an;
    }
    int k = 0;
#pragma unroll
    for (int rr = 0; rr < 6; ++rr) {
        const float wJ = w * J[rr];
#pragma unroll
        for (int c = 0; c <= rr; ++c) acc[k++] += wJ * J[c];
    }
    const float wr = w * res;
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[21 + j] += wr * J[j];
    acc[27] += wr * res;
}
__device__ __forceinline__ void acc_point(const KParams& P, const int32_t* slot, const float (&T)[12], double scale,
                                          float dl, int i, float (&acc)[kNE]) {
    const int s = slot[i];
    if (s < 0) return;
    const float px = P.pts[3 * i], py = P.pts[3 * i + 1], pz = P.pts[3 * i + 2];
    const Slot sl = P.tab[s];             // KDTree path: P.tab = per-point planes, s = i
    double r;
    if (P.kd_res) {
        r = P.kd_res[i];                  // the stored fp64 distance (residuals[i], :374)
    } else {
        float wx, wy, wz;
        transform_pt(T, px, py, pz, wx, wy, wz);
        r = residual_f64(sl, wx, wy, wz);
    }
    acc_terms(P, T, scale, dl, r, px, py, pz, sl, acc);
}
__device__ __forceinline__ void acc_point(const KParams& P, const float (&T)[12], double scale, float dl, int i,
                                          float (&acc)[kNE]) {
    acc_point(P, P.slot, T, scale, dl, i, acc);
}

}  // namespace lo
