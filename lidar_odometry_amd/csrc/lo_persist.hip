// lo_persist.hip — the whole Gauss-Newton loop of one small scan in ONE persistent launch (k_gn).
//
// Reference: IterativeClosestPointOptimizer::optimize, src/optimization/IterativeClosestPointOptimizer.cpp:281-449
// (per iteration: find_correspondences :587-645, the iteration-0 scale :304-316, PKO :318-332 ->
// AdaptiveMEstimator.cpp:243-291, normal equations :345-415, LDLT + SE3 update :417-434, convergence :437-448).
//
// Why: a KITTI scan converges after ~2.4 of its max_iterations = 4 GN iterations, but the launch-per-stage form
// (k_correspond, then per iteration k_pko_t + k_solve_correspond) must enqueue all of them without a host sync; the
// launches after convergence still cost ~4-6 us each on the device timeline (the round-2 in-step trace: 16.6 us per
// scan of early-exit launches).  Here a scan is one launch, and a converged scan's workgroups simply leave.
//
// Roles (grid = G PKO workgroups + (NA + 1) x W candidate workgroups, 256 threads each, all co-resident -- the host
// checks the grid against the occupancy query):
//   A  correspondences: workgroup b < nb searches block b's 256 points at the current pose (correspond_tail, the
//      code of k_correspond / k_solve_correspond) and signals the iteration's A counter;
//   B  every workgroup waits for A, forms n_c / the rank prefix / the scale from the blocks' counts (pko_prefix,
//      every workgroup the same bits); workgroups < G fit the GMM and evaluate their alpha of the JS grid
//      (pko_fit_js), workgroups >= G accumulate one alpha candidate's normal-equation partials (acc_candidate_t),
//      then signal the iteration's B counter;
//   C  every workgroup waits for B, takes the reference's selection (first strict JS minimum), sums the selected
//      candidate's partials (solve_sums) and solves (solve_step) -- the same data and code in every workgroup, so
//      the same pose and the same convergence decision everywhere, with no broadcast; workgroup 0 publishes the
//      GN state and the iteration's log.
// Every per-point term, wave / block tree, partial sum and solve is the multi-launch path's code, so the result is
// bit-identical to it (tests/test_gpu_persist.py).
//
// Hand-offs inside the launch (MI355X_MICROARCH.md "inter-workgroup visibility", the row "one lane of each storing
// workgroup signals by an agent-scope atomic add, the consumer polls with sc1 loads"): every handed-off word is
// stored write-through and loaded past L1 (Mem<true>: global sc1 accesses), every storing wave drains its stores
// (s_waitcnt vmcnt(0)) before the workgroup barrier behind which ONE lane adds to the counter, and one lane polls
// the counter (sc1 loads, s_sleep) before a workgroup barrier.  The JS grid and the candidate partials are
// double-buffered by iteration parity, so a workgroup still reading iteration k's while another writes iteration
// k + 1's cannot collide (a buffer is rewritten only in iteration k + 2, after every workgroup's B(k + 1) arrival).
// Every wait is bounded (2 s, s_memrealtime): a grid that is not co-resident fails with status LO_ERR_HIP instead
// of hanging; the last workgroup to leave re-zeroes the counters for the next launch on the stream.
#include "lo_pko_body.h"
#include "lo_solve.h"

namespace lo {

// sync word layout (per context, zeroed once at creation; the launch's last workgroup re-zeroes what it used)
constexpr int kSyncA = 0;                                // [64] correspondence arrivals per GN iteration
constexpr int kShardB = 8;                               // B arrivals sharded by blockIdx % 8 (~one XCD each, speed only)
constexpr int kSyncB = LO_MAX_ITERS;                     // [64][8] PKO / candidate arrivals per GN iteration
constexpr int kSyncCand = kSyncB + LO_MAX_ITERS * kShardB;   // [kMaxAlpha + 1] per-candidate arrivals (W > 1)
constexpr int kSyncExit = kSyncCand + kMaxAlpha + 1;
constexpr int kSyncTmo = kSyncExit + 1;                  // set by a workgroup whose wait timed out
constexpr int kSyncWords = kSyncTmo + 1;
static_assert(kSyncWords <= kGnSyncWords, "sync buffer");
constexpr unsigned long long kSpinTicks = 200000000ull;   // 2 s of s_memrealtime (100 MHz)

// Diagnostic build only (-DLO_PKO_STAMPS, scripts/gn_phases.py): workgroup 0 stores s_memrealtime (100 MHz) at the
// phase boundaries of GN iterations 0-2 into DevState::dbg: [0] start, then per iteration it at 1 + 5 it + {0: A
// signalled, 1: A waited, 2: B done, 3: B waited, 4: C done}.
#ifdef LO_PKO_STAMPS
#define GN_STAMP(i) do { if (wg == 0 && threadIdx.x == 0 && (i) < 16) st->dbg[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define GN_STAMP(i) do { } while (0)
#endif

// Every storing wave drains its stores, the workgroup meets: the bytes are then visible to whoever sees the signal
// one lane of this workgroup sends next.
__device__ __forceinline__ void gn_drain() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}
__device__ __forceinline__ unsigned gn_add(unsigned* w) {
    return __hip_atomic_fetch_add((g_u32*)(w), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until the sum of counter[0..nshard) reaches target: lanes < nshard of wave 0 poll one shard each (sc1 loads,
// s_sleep between polls), then the workgroup barrier.  false: timed out, or another workgroup timed out.
__device__ __forceinline__ bool gn_wait(unsigned* counter, int nshard, unsigned target, unsigned* tmo, int* s_ok) {
    if (threadIdx.x < kWave) {
        const int lane = threadIdx.x;
        int ok = 1;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            unsigned v = lane < nshard ? Mem<true>::ld(counter + lane) : 0u;
            const unsigned tm = lane == 0 ? Mem<true>::ld(tmo) : 0u;
#pragma unroll
            for (int o = 1; o < kShardB; o <<= 1) v += __shfl_xor(v, o, kWave);
            if (__shfl(v, 0, kWave) >= target) break;
            if (__shfl(tm, 0, kWave) != 0u) { ok = 0; break; }
            if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
                if (lane == 0) Mem<true>::st(tmo, 1u);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: keeps the loads below the poll
        if (lane == 0) *s_ok = ok;
    }
    __syncthreads();
    return *s_ok != 0;
}

// The three phases as separate (non-inlined) functions: each gets its own register allocation -- merged into the
// kernel's loop, the compiler hoisted every phase's loop-invariant addresses and table loads out of the GN loop and
// needed 256 VGPRs (one workgroup per CU; measured 7 % slower than the calls).
// The phases receive the kernel's parameter block as a constant-address-space pointer (the kernarg segment): field
// reads stay scalar loads inside the non-inlined functions (through a generic pointer they became flat vector loads).
typedef const __attribute__((address_space(4))) KParams KParamsC;
#ifndef LO_GN_PHASE
#define LO_GN_PHASE __noinline__
#endif

// One alpha candidate's solved GN step (solve_step's results but n_corr / scale / alpha), [parity][NA + 1] words.
constexpr int kCandWords = kGnCandWords;   // pose[12] | cost | H[21] | g[6] | delta[6] | conv | pad
constexpr int kCandCost = 12, kCandH = 13, kCandG = 34, kCandD = 40, kCandConv = 46;

struct GnLds {
    PkoLds<4> pko;
    double tot[kNE];
    double alpha, scale0;
    float T[12];                                            // the current iteration's pose
    float rec[kCandWords];                                  // a candidate record (packing / the selected one)
    int ok, c;
};

__device__ __forceinline__ CorrOut gn_set(const GnSets& Z, size_t set) {
    const size_t n = static_cast<size_t>(Z.cs_pts);
    return CorrOut{Z.slot + set * n, Z.res + set * n, Z.wmask + set * (n / kWave), Z.cnt + set * (n / kBlock),
                   nullptr, nullptr};
}

// A: find_correspondences (:587-645) at the current pose for blocks wg, wg + NWG, ... (handed-off stores)
__device__ LO_GN_PHASE void gn_phase_a(KParamsC* Pc, int it, int wg, int NWG, GnLds& S) {
    const KParams& P = *(const KParams*)(Pc);
    const int tid = threadIdx.x, n = scan_n(P);
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = S.T[k];
    for (int b = wg; b < P.nb; b += NWG) {
        const int i = b * kBlock + tid;
        float px = 0.0f, py = 0.0f, pz = 0.0f;
        if (i < n) { px = P.pts[3 * i]; py = P.pts[3 * i + 1]; pz = P.pts[3 * i + 2]; }
        correspond_tail<true>(P, T, px, py, pz, i, n, it == 0 ? 1 : 0, b);
    }
}

// One alpha candidate's chain for this iteration (workgroup `part` of the candidate's W): the normal-equation partials
// of its blocks with the candidate's Huber delta; once all W parts have arrived (per-candidate counter, monotonic
// over the iterations), the solve (:417-448) -- every part the same bits -- and, unless it converged, the NEXT
// iteration's correspondences at the candidate's pose for its blocks.  All of it runs while the EM of this
// iteration runs elsewhere, so after the selection the next iteration's correspondences are already there.
__device__ __forceinline__ bool gn_candidate(const KParams& P, const GnArgs A, int it, int c, int part,
                                             const int32_t* slot, double scale, double* acc, float* recs, GnLds& S) {
    const int tid = threadIdx.x;
    const int vb0 = part * A.per, vb1 = min(P.nb_acc, vb0 + A.per);
    double* part_c = acc + static_cast<size_t>(c) * kFuseMaxBlocks * kNE;
    {
        float T[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) T[k] = S.T[k];
        acc_blocks<true>(P, slot, T, scale, cand_delta(P, c), vb0, vb1, part_c);
    }
    unsigned* const cnt = A.sync + kSyncCand + c;
    if (A.W > 1) {
        gn_drain();
        if (tid == 0) gn_add(cnt);
        if (!gn_wait(cnt, 1, static_cast<unsigned>(A.W * (it + 1)), A.sync + kSyncTmo, &S.ok)) return false;
    } else {
        gn_drain();                                          // this workgroup's own partials, read back through L2
    }
    solve_sums<kBlock, true>(part_c, P.nb_acc, S.tot);
    if (tid == 0) {
        float T[12], Tn[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) T[k] = S.T[k];
        lo_iter_log lg;
        const bool conv = solve_step(P, S.tot, T, Tn, &lg);
#pragma unroll
        for (int q = 0; q < 12; ++q) S.rec[q] = Tn[q];
        S.rec[kCandCost] = lg.cost;
#pragma unroll
        for (int q = 0; q < 21; ++q) S.rec[kCandH + q] = lg.H[q];
#pragma unroll
        for (int q = 0; q < 6; ++q) { S.rec[kCandG + q] = lg.g[q]; S.rec[kCandD + q] = lg.delta[q]; }
        S.rec[kCandConv] = conv ? 1.0f : 0.0f;
        S.rec[kCandConv + 1] = 0.0f;
    }
    __syncthreads();
    if (part == 0 && tid < kCandWords) Mem<true>::st(recs + static_cast<size_t>(c) * kCandWords + tid, S.rec[tid]);
    if (S.rec[kCandConv] == 0.0f && it + 1 < P.max_iters) {
        float Tn[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) Tn[k] = S.rec[k];
        const CorrOut O = gn_set(A.sets, static_cast<size_t>((it + 1) & 1) * (P.NA + 1) + c);
        const int n = scan_n(P);
        for (int b = part * A.per; b < min(P.nb, (part + 1) * A.per); ++b) {
            const int i = b * kBlock + tid;
            float px = 0.0f, py = 0.0f, pz = 0.0f;
            if (i < n) { px = P.pts[3 * i]; py = P.pts[3 * i + 1]; pz = P.pts[3 * i + 2]; }
            correspond_tail<true>(P, O, Tn, px, py, pz, i, n, 0, b);
        }
    }
    return true;
}

// B: n_c / prefix / scale in every workgroup (from this iteration's correspondence set), then the GMM + this
// workgroup's JS alpha (wg < G) or a part of one candidate's chain (wg >= G).  Returns n_c (the caller stops the
// scan below min_correspondence_points), or -1 when a candidate's wait timed out.
__device__ LO_GN_PHASE int gn_phase_b(KParamsC* Pc, const GnArgs A, int it, int wg, const ScanBufs cur, double* js,
                                      double* acc, float* recs, GnLds& S, int* s_pre) {
    const KParams& P = *(const KParams*)(Pc);
    const int tid = threadIdx.x, G = A.G;
    PrefixLoads pl;
    if (tid < kWave) {
        prefix_loads<true>(P, cur, it, pl);
        pl.sc = S.scale0;                                    // later iterations: the iteration-0 scale (:304-316)
    }
    PkoPrefetch pf;                                          // in flight with the prefix (as pko_body's)
    if (wg < G) pko_prefetch<4>(P, wg, G, pf, S.pko);
    int nc;
    double sc;
    pko_prefix<4>(P, cur, it, wg == 0, s_pre, nc, sc, S.pko.wm, &pl);
    if (it == 0 && tid == 0) S.scale0 = sc;
    if (nc < P.min_corr) return nc;                          // :298-302 -- every workgroup reads the same counts
    if (wg >= G) {
        const int c = (wg - G) / A.W, part = (wg - G) - c * A.W;
        if (c <= P.NA && !gn_candidate(P, A, it, c, part, cur.slot, sc, acc, recs, S)) return -1;
    } else {
        if (wg == 0 && tid == 0) P.st->n_corr = nc;
        ScanBufs Bj = cur;
        Bj.js = js;
        pko_fit_js<4, false, true>(P, Bj, wg, G, nc, sc, pf, s_pre, S.pko.wm, S.pko, nullptr);
    }
    return nc;
}

// C: the reference's selection (first strict JS minimum, AdaptiveMEstimator.cpp:256-275) and the selected
// candidate's solved step (formed in phase B).  Workgroup 0 publishes the GN state and the iteration's log.  Returns
// the selected candidate, with its convergence test in S.rec (the same in every workgroup).
__device__ LO_GN_PHASE int gn_phase_c(KParamsC* Pc, int it, int wg, int nc, const double* js, const float* recs,
                                      GnLds& S) {
    const KParams& P = *(const KParams*)(Pc);
    const int tid = threadIdx.x;
    DevState* st = P.st;
    if (tid < kWave) {
        const int bi = pko_select_index<true>(P, js);
        const int c = bi > 0 ? bi - 1 : P.NA;
        if (tid < kCandWords) S.rec[tid] = Mem<true>::ld(recs + static_cast<size_t>(c) * kCandWords + tid);
        if (tid == 0) { S.alpha = bi > 0 ? P.alphas[bi] : P.min_scale; S.c = c; }
    }
    __syncthreads();
    if (wg == 0 && tid == 0) {
        lo_iter_log& L = st->logs[it];
#pragma unroll
        for (int q = 0; q < 12; ++q) { st->pose[q] = S.rec[q]; L.pose[q] = S.rec[q]; }
        L.n_corr = nc;
        L.scale = S.scale0;
        L.alpha = S.alpha;
        L.cost = S.rec[kCandCost];
#pragma unroll
        for (int q = 0; q < 21; ++q) L.H[q] = S.rec[kCandH + q];
#pragma unroll
        for (int q = 0; q < 6; ++q) { L.g[q] = S.rec[kCandG + q]; L.delta[q] = S.rec[kCandD + q]; }
        st->alpha = S.alpha;
        st->iter = it + 1;
        if (S.rec[kCandConv] != 0.0f) st->done = 1;
    }
    if (tid < 12) S.T[tid] = S.rec[tid];
    __syncthreads();
    return S.c;
}

__global__ __launch_bounds__(kBlock, 3) void k_gn(KParams P, GnArgs A) {
    const int wg = blockIdx.x, NWG = static_cast<int>(gridDim.x), tid = threadIdx.x;
    DevState* st = P.st;
    extern __shared__ int s_pre[];                           // nb ints: exclusive prefix of the block counts
    __shared__ GnLds S;
    // P is the first kernel argument: offset 0 of the kernarg segment (taking &P would address a private copy)
    KParamsC* const Pc = (KParamsC*)(__builtin_amdgcn_kernarg_segment_ptr());
    if (tid < 12) S.T[tid] = P.T0[tid];
    if (tid == 0) S.scale0 = 0.0;
    if (wg == 0) {                                           // the fresh GN state (k_init / k_correspond's reset)
        if (tid < 12) st->pose[tid] = P.T0[tid];
        if (tid == 0) {
            st->scale = 1.0;
            st->alpha = P.robust_delta;
            st->n_corr = 0;
            st->iter = 0;
            st->done = 0;
            st->status = LO_OK;
        }
    }
    __syncthreads();
    GN_STAMP(0);
    const int nCorr = min(P.nb, NWG);
    const size_t js_set = static_cast<size_t>(P.NA) + 1;
    const size_t acc_set = js_set * kFuseMaxBlocks * kNE;
    const size_t rec_set = js_set * kCandWords;
    unsigned* const tmo = A.sync + kSyncTmo;
    ScanBufs cur = own_bufs(P);                              // iteration 0: the context's own correspondence buffers
    bool ok = true;
    for (int it = 0; it < P.max_iters; ++it) {
        const int par = it & 1;
        double* js = P.js + par * js_set;
        double* acc = P.acc_part + par * acc_set;
        float* recs = A.cand + par * rec_set;
        unsigned* const cB = A.sync + kSyncB + it * kShardB;
        if (it == 0 && !A.skip_corr0) {
            unsigned* const cA = A.sync + kSyncA;
            if (wg < nCorr) {
                gn_phase_a(Pc, it, wg, NWG, S);
                gn_drain();
                if (tid == 0) gn_add(cA);
            }
            GN_STAMP(1);
            if (!(ok = gn_wait(cA, 1, static_cast<unsigned>(nCorr), tmo, &S.ok))) break;
        }
        GN_STAMP(2 + 5 * it);
        const int nc = gn_phase_b(Pc, A, it, wg, cur, js, acc, recs, S, s_pre);
        GN_STAMP(3 + 5 * it);
        if (nc < 0) { ok = false; break; }
        if (nc < P.min_corr) {
            if (wg == 0 && tid == 0) { st->status = LO_INSUFFICIENT; st->done = 1; st->n_corr = nc; }
            break;
        }
        gn_drain();
        if (tid == 0) gn_add(cB + (wg & (kShardB - 1)));
        if (!(ok = gn_wait(cB, kShardB, static_cast<unsigned>(NWG), tmo, &S.ok))) break;
        GN_STAMP(4 + 5 * it);
        const int c = gn_phase_c(Pc, it, wg, nc, js, recs, S);
        GN_STAMP(5 + 5 * it);
        if (S.rec[kCandConv] != 0.0f) break;
        // the next iteration reads the selected candidate's correspondences (its pose is S.T now)
        const CorrOut O = gn_set(A.sets, static_cast<size_t>((it + 1) & 1) * (P.NA + 1) + c);
        cur.slot = O.slot;
        cur.res = O.res;
        cur.wmask = O.wmask;
        cur.blk_cnt = O.blk_cnt;
    }
    if (!ok && wg == 0 && tid == 0) {                        // a wait timed out: the grid was not co-resident
        st->status = LO_ERR_HIP;
        st->done = 1;
    }
    // leave: the last workgroup out re-zeroes the counters for the next launch on this stream
    gn_drain();
    if (tid < kWave) {
        unsigned prev = 0;
        if (tid == 0) prev = gn_add(A.sync + kSyncExit);
        prev = __shfl(prev, 0, kWave);
        if (prev == static_cast<unsigned>(NWG - 1)) {
            for (int w = tid; w < kSyncWords; w += kWave) Mem<true>::st(A.sync + w, 0u);
        }
    }
}

}  // namespace lo
