// lo_kernels.hip — HIP kernels of the point-to-plane ICP hot path for gfx950 (MI355X / CDNA4).
//
// One Gauss-Newton iteration of IterativeClosestPointOptimizer::optimize
// (reference src/optimization/IterativeClosestPointOptimizer.cpp:281-449) is built from these launches on one
// stream (small scans with PKO: k_pko also accumulates every alpha candidate's normal equations and the solve runs
// fused with the next iteration's correspondences, k_solve_correspond -- two launches per iteration; see
// launch_gn_tail / enqueue_optimize in lo_icp.hip):
//   k_correspond  per point: transform, L1 surfel probe, fp64 residual, accept r <= max_corr
//                 (find_correspondences :587-645); per-wave validity ballots; iteration 0 also the
//                 per-block residual sum / M2 for the normalisation scale (:304-316)
//   k_pko         (lo_pko.hip) correspondence count, scale, the reference's PKO sample selection, GMM fit
//                 and the JS-divergence alpha grid (AdaptiveMEstimator.cpp:243-485, :710-787)
//   k_accumulate  per correspondence: Huber weight, residual, Jacobian, 21+6+1 partial sums; wave shuffle
//                 + LDS tree to one 28-double partial per block (:345-410)
//   k_solve       one workgroup: fixed-order fp64 sum of block partials, pivoted LDLT (:418),
//                 SE3 right-update with SO(3) re-projection (:422-434), convergence flag (:437-448)
// Every kernel first reads DevState::done, so the whole max_iterations sequence is enqueued once and
// converged / failed scans fall through without a host round trip.
//
// Compiled with -ffp-contract=off: the correspondence set and the fp64 residuals are bit-identical to the
// reference's fp32/fp64 expressions (DESIGN.md "fp order").  Sums are fixed-order trees (run-to-run
// deterministic), not the reference's sequential order.
#include "lo_blocksort.h"
#include "lo_device.h"
#include "lo_math.h"
#include "lo_solve.h"

#include <cfloat>

namespace lo {

// ====================================================================================================
// k_correspond
// ====================================================================================================
// init: first launch of a scan.  The GN state reset (k_init's job) is folded in here -- the pose comes from
// the kernel argument (T0 / T0p), block 0 writes the fresh DevState that the later kernels of the scan read.
// The point load is issued before the DevState loads (done flag, pose) so the three latencies overlap
// instead of serialising at the start of every wave.
__device__ __forceinline__ void correspond_body(const KParams& P, int with_stats, int init, int blk) {
    // timing (P.span, lo_set_stage_timing / lo_bench_kernel 5): the launch's own execution span, without the dispatch
    // latency a pair of HIP events around it includes -- the first blocks' starts and the last blocks' ends, plain
    // stores (one address hit by every block's atomic serialises: ~80 us at 1M points)
    if (P.span && threadIdx.x == 0 && blk < kSpanStarts)
        P.span[blk] = static_cast<unsigned long long>(__builtin_amdgcn_s_memrealtime());
    const int i = blk * kBlock + threadIdx.x;
    const int n = scan_n(P);
    float px = 0.0f, py = 0.0f, pz = 0.0f;
    if (i < n) { px = P.pts[3 * i]; py = P.pts[3 * i + 1]; pz = P.pts[3 * i + 2]; }
    const DevState* cst = P.st;
    const int done = cst->done;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = cst->pose[k];
    if (!init && done) return;
    scan_pose(P, init, blk, T);
    const uint64_t key = correspond_tail(P, T, px, py, pz, i, n, with_stats, blk);
    if (P.presort) presort_block(P.presort, blk, key);      // iteration 0, reference-exact mode (uniform branch)
    if (P.span) {                                           // after every thread's stores of the block have issued
        const int e = blk - (P.nb > kSpanEnds ? P.nb - kSpanEnds : 0);
        __syncthreads();
        if (threadIdx.x == 0 && e >= 0) P.span[kSpanStarts + e] = static_cast<unsigned long long>(__builtin_amdgcn_s_memrealtime());
    }
}

// XCD-aware block order: the hardware hands consecutive workgroups to the 8 XCDs round-robin; logical block
// xcd_block(h) gives XCD x (= h % 8) one contiguous run of the scan's blocks, so spatially coherent points (scans in
// acquisition order) probe the same surfel-table lines through one L2 instead of eight.  A bijection on [0, nb).
__device__ __forceinline__ int xcd_block(int h, int nb) {
    constexpr int kXcd = 8;
    const int q = nb / kXcd, r = nb % kXcd, x = h % kXcd, k = h / kXcd;
    return x < r ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
}

__global__ __launch_bounds__(kBlock) void k_correspond(KParams P, int with_stats) {
    correspond_body(P, with_stats, P.init, xcd_block(blockIdx.x, gridDim.x));
}

// Batched launch (lo_batch_*): blockIdx.y = job (one context each: own scan, map and GN state); the grid is
// sized for the largest job and a job's surplus blocks leave before touching any of its buffers.
// Batched: the (block, job) grid is linearised and put in XCD-aware order, so each XCD takes whole jobs and a
// job's surfel table is cached by one L2.
__global__ __launch_bounds__(kBlock) void k_correspond_b(const KParams* __restrict__ PB, int with_stats, int init) {
    const int total = static_cast<int>(gridDim.x * gridDim.y);
    const int lin = xcd_block(static_cast<int>(blockIdx.x + blockIdx.y * gridDim.x), total);
    const int job = lin / static_cast<int>(gridDim.x), blk = lin - job * static_cast<int>(gridDim.x);
    const KParams& P = PB[job];
    if (blk >= P.nb) return;
    correspond_body(P, with_stats, init, blk);
}

// ====================================================================================================
// k_accumulate
// ====================================================================================================
template <int NT>
__device__ void solve_tail(const KParams& P, int it, int ne_only, const double* part_src, int nrows);

// fuse: 0 = partials only, 1 = the last block to finish also runs the GN solve / update (k_solve's job),
// 2 = the last block writes the summed normal equations (lo_build_normal_equations)
__device__ __forceinline__ void accumulate_body(const KParams& P, int it, int fuse, int blk, int nblk) {
    DevState* st = P.st;
    if (st->done) return;
    __shared__ float s_acc[kWavesPerBlock][kNE];
    __shared__ double s_alpha;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // Huber delta of this iteration: argmin of the JS grid k_pko wrote (PKO), else robust_loss_delta
    if (wid == 0) {
        const double a = P.alpha_given ? P.st->alpha : (P.use_pko ? pko_select_alpha(P) : P.robust_delta);
        if (lane == 0) {
            s_alpha = a;
            if (blk == 0 && !P.alpha_given) P.st->alpha = a;
        }
    }
    __syncthreads();
    float acc[kNE];
#pragma unroll
    for (int k = 0; k < kNE; ++k) acc[k] = 0.0f;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
    const double scale = st->scale;
    const float dl = static_cast<float>(s_alpha);
    // grid-stride (at most kAccBlocks blocks): per-thread fp32 sums of <= 4 points at 1M, then the same
    // wave / block trees; the partial count k_solve reduces stays <= kAccBlocks
    const int n = scan_n(P);
    for (int i = blk * kBlock + tid; i < n; i += P.nb_acc * kBlock) acc_point(P, T, scale, dl, i, acc);
    wave_totals_f32<kNE>(acc, s_acc[wid]);
    __syncthreads();
    if (tid < kNE) {
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < kWavesPerBlock; ++w) v += static_cast<double>(s_acc[w][tid]);
        P.blk_part[static_cast<size_t>(blk) * kNE + tid] = v;
    }
    if (fuse == 0) return;
    // last-block-done: release the partials at agent scope (the 8 XCDs have separate L2s), count arrivals;
    // the block that arrives last acquires and reduces them in fixed block order -- one launch fewer per
    // GN iteration, same deterministic sum as a separate k_solve
    __shared__ int s_last;
    __threadfence();
    __syncthreads();
    if (tid == 0) s_last = (atomicAdd(&st->acc_arrive, 1u) == static_cast<unsigned>(nblk - 1)) ? 1 : 0;
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    if (tid == 0) st->acc_arrive = 0;
    solve_tail<kBlock>(P, it, fuse == 2, P.blk_part, P.nb_acc);
}

__global__ __launch_bounds__(kBlock) void k_accumulate(KParams P, int it, int fuse) {
    accumulate_body(P, it, fuse, blockIdx.x, gridDim.x);
}

// Batched launch for batches with a large job (> kFuseMaxBlocks blocks): blockIdx.y = job, partials only;
// k_solve_b reduces and solves every job.
__global__ __launch_bounds__(kBlock) void k_accumulate_b(const KParams* __restrict__ PB, int it) {
    const KParams& P = PB[blockIdx.y];
    if (static_cast<int>(blockIdx.x) >= P.nb_acc) return;
    accumulate_body(P, it, 0, blockIdx.x, P.nb_acc);
}

// ====================================================================================================
// k_solve
// ====================================================================================================
template <int NT>
__device__ void solve_tail(const KParams& P, int it, int ne_only, const double* part_src, int nrows) {
    DevState* st = P.st;
    __shared__ double tot[kNE];
    solve_sums<NT>(part_src, nrows, tot);
    if (threadIdx.x != 0) return;
    if (ne_only) {
        int k = 0;
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c <= r; ++c) { st->H_out[r * 6 + c] = tot[k]; st->H_out[c * 6 + r] = tot[k]; ++k; }
        for (int j = 0; j < 6; ++j) st->g_out[j] = tot[21 + j];
        st->cost_out = tot[27];
        return;
    }
    float pn[12];
    solve_core(P, it, tot, st->pose, pn, true);
}

// Standalone solve over all block partials (lo_bench_kernel; the GN loop fuses it into k_accumulate)
__global__ __launch_bounds__(kSolveThreads) void k_solve(KParams P, int it, int ne_only) {
    if (P.st->done) return;
    solve_tail<kSolveThreads>(P, it, ne_only, P.blk_part, P.nb_acc);
}

// Solve from the speculative normal equations (single scans with nb_acc <= kFuseMaxBlocks): the candidate of
// the selected alpha (acc_candidate, lo_pko.hip) holds the same per-block partials the fused k_accumulate would
// have formed, reduced here with the same solve_tail<kBlock> pattern -- bit-identical, one launch fewer.
__global__ __launch_bounds__(kBlock) void k_solve_pick(KParams P, int it) {
    DevState* st = P.st;
    const int done = st->done;                   // loaded together with the JS grid
    __shared__ int s_c, s_skip;
    int bi = 0;
    if (threadIdx.x < kWave) bi = pko_select_index(P);
    if (threadIdx.x == 0) {
        s_skip = done;
        if (!done) {
            s_c = bi > 0 ? bi - 1 : P.NA;
            st->alpha = bi > 0 ? P.alphas[bi] : P.min_scale;
        }
    }
    __syncthreads();
    if (s_skip) return;
    solve_tail<kBlock>(P, it, 0, P.acc_part + static_cast<size_t>(s_c) * kFuseMaxBlocks * kNE, P.nb_acc);
}

// The solve of GN iteration it fused with the correspondence search of iteration it + 1 (single small scans with
// PKO, surfel path): every block reduces the selected candidate's partials and solves redundantly -- same data,
// same code, so the same pose in every block -- then searches its 256 points with the new pose; block 0
// publishes the GN state.  The old pose is read from the previous iteration's log (the initial pose for it = 0),
// which no block of this launch writes.  One launch per GN iteration fewer than k_solve_pick + k_correspond.
__global__ __launch_bounds__(kBlock) void k_solve_correspond(KParams P, int it) {
    DevState* st = P.st;
    const int tid = threadIdx.x, blk = blockIdx.x;
    // the done flag, the points and the JS grid are loaded together (one round trip, not two); a converged scan
    // leaves after it without writing anything
    const int done = st->done;
    const int i = blk * kBlock + tid;
    const int n = scan_n(P);
    float px = 0.0f, py = 0.0f, pz = 0.0f;       // in flight during the solve
    if (i < n) { px = P.pts[3 * i]; py = P.pts[3 * i + 1]; pz = P.pts[3 * i + 2]; }
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
    if (s_done) return;                          // converged: the later launches of the scan see DevState::done
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = s_T[k];
    correspond_tail(P, T, px, py, pz, i, n, 0, blk);
}

// The selection of GN iteration it (pko_select_index: the reference's first strict JS minimum,
// AdaptiveMEstimator.cpp:256-275) applied to the candidates the PKO launch already solved (acc_candidate with
// P.cand_rec): the selected record is the iteration's pose, log and convergence test (:417-448), block 0 publishes
// the GN state, and with CORR every block then searches its 256 points at the new pose for iteration it + 1 -- the
// fp64 solve is no longer between the EM's end and the next correspondence search.  Same record = same bits as
// k_solve_pick / k_solve_correspond.
// Scan pipeline, the main part's last pick (P.hold) when the scan goes on: every block writes its correspondences
// back (agent release after its waves' stores have drained) and counts itself in; the last block tells the tail
// stream that the main part is done (fin[1] = seq).  k_wait_seq heads the tail and the tail's next kernel starts with
// an acquire.  Nothing here waits: a wait may only depend on work submitted before it, or two streams that share a
// hardware queue would deadlock.
__device__ __forceinline__ void signal_main(const KParams& P) {
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_last = __hip_atomic_fetch_add(P.fin + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (threadIdx.x != 0 || !s_last) return;
    __hip_atomic_store(P.fin + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(P.fin + 1, P.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool CORR>
__device__ __forceinline__ void pick_body(const KParams& P, int it) {
    const int tid = threadIdx.x, blk = blockIdx.x;
    const int i = blk * kBlock + tid;
    const int n = scan_n(P);
    float px = 0.0f, py = 0.0f, pz = 0.0f;
    // tail-stream launches (scan pipeline) read the caller's points only once the scan is known to go on: they
    // may run after the caller has already taken the final result and reused or freed that buffer
    if (CORR && !P.tail && i < n) { px = P.pts[3 * i]; py = P.pts[3 * i + 1]; pz = P.pts[3 * i + 2]; }
    __shared__ float s_rec[kCandWords];
    bool conv = false;
    if (!pick_select(P, it, s_rec, &conv)) return;
    if (!CORR || conv) return;                    // converged: the later launches of the scan see DevState::done
    if (P.tail && i < n) { px = P.pts[3 * i]; py = P.pts[3 * i + 1]; pz = P.pts[3 * i + 2]; }
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = s_rec[k];
    correspond_tail(P, T, px, py, pz, i, n, 0, blk);
    if (P.hold) signal_main(P);
}
__global__ __launch_bounds__(kBlock) void k_pick_correspond(KParams P, int it) { pick_body<true>(P, it); }
__global__ __launch_bounds__(kBlock) void k_pick(KParams P, int it) { pick_body<false>(P, it); }

// Batched solve (jobs with more than kFuseMaxBlocks accumulate blocks present): one block per job, with the
// partial-sum pattern the single-scan path uses for that job's size, so every job stays bit-identical to it.
__global__ __launch_bounds__(kSolveThreads) void k_solve_b(const KParams* __restrict__ PB, int it) {
    const KParams& P = PB[blockIdx.x];
    if (P.st->done) return;
    if (P.nb_acc <= kFuseMaxBlocks) solve_tail<kBlock>(P, it, 0, P.blk_part, P.nb_acc);
    else solve_tail<kSolveThreads>(P, it, 0, P.blk_part, P.nb_acc);
}

// Batched accumulate + solve for small jobs (nb_acc <= kFuseMaxBlocks): ONE workgroup of 8 waves per job walks
// the job's 256-point blocks two at a time (wave w takes block 2r + w/4, its quarter w%4), so each point, wave
// sum and per-block fp64 partial is formed exactly as in the multi-block launch; the partials stay in LDS and the
// same workgroup solves.  No inter-workgroup hand-off: no atomics and no agent-scope fences (whose L2 write-back
// and invalidate per workgroup dominated the multi-block form once thousands of workgroups were in flight).
// SOLVE = false (the default batch form): the per-block partials go to the job's blk_part and k_solve_b1 solves --
// the fp64 solve's registers then size neither launch (fused, the solve pins this 8-wave kernel at 128 VGPRs plus
// scratch spills, 2 workgroups per CU).
constexpr int kAcc1Threads = 512;
template <bool SOLVE>
__global__ __launch_bounds__(kAcc1Threads) void k_accumulate_b1(const KParams* __restrict__ PB, int it) {
    const KParams& P = PB[blockIdx.y];
    DevState* st = P.st;
    if (st->done) return;
    constexpr int kW = kAcc1Threads / kWave;           // 8 waves = 2 virtual blocks per pass
    __shared__ float s_acc[kW][kNE];
    __shared__ double s_part[kFuseMaxBlocks * kNE];
    __shared__ double s_alpha;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (wid == 0) {
        const double a = P.use_pko ? pko_select_alpha(P) : P.robust_delta;
        if (lane == 0) { s_alpha = a; st->alpha = a; }
    }
    __syncthreads();
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
    const double scale = st->scale;
    const float dl = static_cast<float>(s_alpha);
    const int n = scan_n(P), nb = P.nb_acc;
    for (int vb0 = 0; vb0 < nb; vb0 += kW / kWavesPerBlock) {
        const int vb = vb0 + wid / kWavesPerBlock;
        const int i = vb * kBlock + (wid % kWavesPerBlock) * kWave + lane;
        float acc[kNE];
#pragma unroll
        for (int k = 0; k < kNE; ++k) acc[k] = 0.0f;
        if (vb < nb && i < n) acc_point(P, T, scale, dl, i, acc);
        wave_totals_f32<kNE>(acc, s_acc[wid]);
        __syncthreads();
        if (tid < kW / kWavesPerBlock * kNE) {
            const int q = tid / kNE, k = tid - q * kNE;
            if (vb0 + q < nb) {
                double v = 0.0;
#pragma unroll
                for (int w = 0; w < kWavesPerBlock; ++w) v += static_cast<double>(s_acc[q * kWavesPerBlock + w][k]);
                s_part[(vb0 + q) * kNE + k] = v;
            }
        }
        __syncthreads();
    }
    if (SOLVE) {
        solve_tail<kBlock>(P, it, 0, s_part, nb);
    } else {
        for (int k = tid; k < nb * kNE; k += kAcc1Threads) P.blk_part[k] = s_part[k];
    }
}
template __global__ void k_accumulate_b1<true>(const KParams*, int);
template __global__ void k_accumulate_b1<false>(const KParams*, int);

// The solve after k_accumulate_b1<false>: one 256-thread workgroup per job, the same solve_tail<kBlock> over the same
// partials as the fused form (bit-identical), with a 256-thread register budget.
__global__ __launch_bounds__(kBlock) void k_solve_b1(const KParams* __restrict__ PB, int it) {
    const KParams& P = PB[blockIdx.x];
    if (P.st->done) return;
    solve_tail<kBlock>(P, it, 0, P.blk_part, P.nb_acc);
}

// ====================================================================================================
// k_map_patch: in-place surfel table patch (lo_map_patch_surfels).  One thread per changed L1 voxel (keys unique
// within a patch): an upsert finds its key and overwrites the payload, or claims the first EMPTY slot of its probe
// sequence with a CAS on the key (tombstones are never reused, so the key cannot sit past an empty slot); an erase
// turns its slot into a tombstone, which lookup_surfel probes past (never equal to a packed key, never empty).
// The ICP kernels read the table only after this launch (stream order), so payload stores need no ordering.
// ====================================================================================================
struct MapPatchRec {
    uint64_t key;
    float n[3];
    float c[3];
    uint32_t op;
    uint32_t pad;
};

__device__ void patch_slot(Slot* tab, uint32_t log2cap, const MapPatchRec& r) {
    const uint32_t mask = (1u << log2cap) - 1u;
    uint32_t h = hash_slot(r.key, log2cap);
    for (uint32_t p = 0; p <= mask; ++p) {
        unsigned long long* kp = reinterpret_cast<unsigned long long*>(&tab[h].key);
        unsigned long long k = __hip_atomic_load(kp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == r.key) {
            if (r.op == 0) {
                __hip_atomic_store(kp, static_cast<unsigned long long>(kTombKey), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                for (int a = 0; a < 3; ++a) { tab[h].n[a] = r.n[a]; tab[h].c[a] = r.c[a]; }
            }
            return;
        }
        if (k == kEmptyKey) {
            if (r.op == 0) return;                           // not present (the host mirror said it was)
            const unsigned long long prev = atomicCAS(kp, static_cast<unsigned long long>(kEmptyKey),
                                                      static_cast<unsigned long long>(r.key));
            if (prev == kEmptyKey) {
                for (int a = 0; a < 3; ++a) { tab[h].n[a] = r.n[a]; tab[h].c[a] = r.c[a]; }
                return;
            }
            continue;                                        // another insert took the slot: look at it again
        }
        h = (h + 1u) & mask;
    }
}

__global__ __launch_bounds__(kBlock) void k_map_patch(Slot* tab, uint32_t log2cap, const MapPatchRec* rec, int n) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    patch_slot(tab, log2cap, rec[i]);
}

// k_surfel_fit: the deferred refits of a host map's touched L1 voxels (VoxelMap.cpp:211-243, surfel_fit in lo_math.h,
// the host's own code), one thread per voxel: result back to the host map, and the table patched in place -- the
// surfel upserted, or erased when the planarity test fails (:239-247).
struct FitJob {
    uint64_t key;
    int32_t off, m;
};
struct FitOut {
    float n[3], c[3], planarity;
    uint32_t pad;
};
__global__ __launch_bounds__(kBlock) void k_surfel_fit(const FitJob* jobs, const float* cs, int n, float thr, Slot* tab,
                                                       uint32_t log2cap, FitOut* out) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const FitJob J = jobs[i];
    float cen[3], U[3][3];
    const float pl = surfel_fit(cs + 3 * static_cast<size_t>(J.off), J.m, cen, U);
    FitOut o;
    for (int a = 0; a < 3; ++a) { o.n[a] = U[a][2]; o.c[a] = cen[a]; }
    o.planarity = pl;
    o.pad = 0;
    out[i] = o;
    MapPatchRec r;
    r.key = J.key;
    r.op = (pl > thr) ? 0u : 1u;                        // NaN planarity keeps the surfel, as the host comparison
    r.pad = 0;
    for (int a = 0; a < 3; ++a) { r.n[a] = o.n[a]; r.c[a] = o.c[a]; }
    patch_slot(tab, log2cap, r);
}

// ====================================================================================================
// k_init: reset the GN state for a new scan.  The initial pose travels as a kernel argument, so any
// number of scans can be enqueued back to back without a host staging buffer.
// ====================================================================================================
struct Pose12 { float v[12]; };

__global__ void k_init(DevState* st, Pose12 T, double scale, double alpha) {
    if (threadIdx.x < 12) st->pose[threadIdx.x] = T.v[threadIdx.x];
    if (threadIdx.x == 0) {
        st->scale = scale;
        st->alpha = alpha;
        st->n_corr = 0;
        st->iter = 0;
        st->done = 0;
        st->status = LO_OK;
        st->acc_arrive = 0;
        st->kd_unres_n = 0;
        st->inliers = 0;
        st->kd_tie = 0;
    }
}

// Scan pipeline (lo_set_pipeline), both bounded by wait_word:
//   k_wait_seq   heads a scan's tail on the tail stream: the main part is done (fin[1] >= seq, signal_main) or the
//                scan is already final (fin[0] >= seq: its tail launches only leave early);
//   k_wait_final follows the tail on the context stream: holds it until the scan's result is final (fin[0] >= seq).
// Host submission order is main part, tail, k_wait_final: every wait depends only on work submitted before it, so
// the two streams may share one hardware queue (they then simply run in order).  What breaks the device-side waits is a
// dispatcher that serialises the two queues OUT of submission order (rocprofv3 counter collection runs one dispatch
// at a time and can take the context stream's k_wait_final before the tail stream's launches: the wait then waits for
// work that cannot start until it ends).  A wait that times out -- or finds the pipeline already broken -- marks the
// scan LO_ERR_PIPELINE and sets the sticky broken word on the device (fin[3]: every later tail launch leaves without
// touching the context's buffers, every later wait gives up at once) and in pinned host memory (hbroken: the host turns
// the pipeline off at its next enqueue and re-runs a synchronous call's scan on one stream).
__device__ __forceinline__ void pipe_fail(uint32_t* fin, uint32_t* hbroken, uint32_t seq, DevState* st) {
    st->status = LO_ERR_PIPELINE;
    __hip_atomic_store(fin + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (hbroken) __hip_atomic_store(hbroken, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_wait_seq(uint32_t* fin, uint32_t seq, DevState* st, uint32_t* hbroken, unsigned long long bound) {
    if (threadIdx.x != 0) return;
    // bound 0 (LO_PIPE_FAIL_AT, tests): the timeout path taken without waiting
    if (bound == 0 || !wait_word2(fin, fin + 1, seq, fin + 3, bound)) pipe_fail(fin, hbroken, seq, st);
}
__global__ void k_wait_final(uint32_t* fin, uint32_t seq, DevState* st, uint32_t* hbroken, unsigned long long bound) {
    if (threadIdx.x != 0) return;
    if (!wait_word(fin, seq, fin + 3, bound)) pipe_fail(fin, hbroken, seq, st);
}

// Copy the current pose + status into a caller buffer (16 floats: pose[12], status, iterations, n_corr, 0).
__global__ void k_export_pose(const DevState* st, float* out) {
    const int t = threadIdx.x;
    if (t < 12) out[t] = st->pose[t];
    if (t == 12) out[12] = static_cast<float>(st->status);
    if (t == 13) out[13] = static_cast<float>(st->iter);
    if (t == 14) out[14] = static_cast<float>(st->n_corr);
    if (t == 15) out[15] = 0.0f;
}

// Batched result export: one record per job (lo_batch_result reads them with one copy).
__global__ void k_export_batch(const KParams* __restrict__ PB, lo_batch_rec* out) {
    const DevState* st = PB[blockIdx.x].st;
    lo_batch_rec& R = out[blockIdx.x];
    const int t = threadIdx.x;
    if (t < 12) R.pose[t] = st->pose[t];
    if (t == 12) R.status = st->status;
    if (t == 13) R.iterations = st->iter;
    if (t == 14) R.n_corr = st->n_corr;
    if (t == 15) R.alpha = st->alpha;
    if (t == 16) R.initial_cost = st->iter > 0 ? st->logs[0].cost : 0.0f;
    if (t == 17) R.final_cost = st->iter > 0 ? st->logs[min(st->iter, LO_MAX_ITERS) - 1].cost : 0.0f;
}

}  // namespace lo

