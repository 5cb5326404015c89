// lo_lookahead.hip — two Gauss-Newton iterations per launch for small single scans with PKO (surfel path).
//
// A KITTI-size scan spends ~90 % of optimize() in the PKO's strictly sequential EM (AdaptiveMEstimator.cpp:294-485),
// one per GN iteration, and iteration k + 1's EM needs iteration k's Huber delta alpha_k.  But alpha_k is one of
// only NA + 1 values (the JS grid's alphas, or min_scale when no JS cost is finite), so iteration k + 1 can be run
// for EVERY candidate while iteration k's EM runs.  One launch k_la(k) holds:
//   main workgroups (G = one per alpha, as k_pko_t): iteration k's PKO on the current correspondences -> JS grid;
//   chain workgroups (one per candidate c): iteration k's normal equations with delta_c, solve -> pose_{k+1}^c,
//     correspondences at pose_{k+1}^c, iteration k+1's whole PKO (count, sample, k-means, EM, JS grid) ->
//     alpha_{k+1}^c, normal equations + solve -> pose_{k+2}^c, and the correspondences at pose_{k+2}^c that the
//     next launch's main workgroups will use.
// The next launch (or k_la_finish) takes c* = argmin of the main JS grid (the reference's selection,
// AdaptiveMEstimator.cpp:256-275) and publishes candidate c*'s two iterations.  Every chain step is the code of the
// one-iteration-at-a-time path (acc_point, wave / block / solve_sums trees, solve_step, pko_body, the correspondence
// tail), so the published iterations are bit-identical to it; the EM chains of iterations k and k+1 overlap, which
// halves the EMs on a scan's critical path (2 launches for 3-4 iterations instead of 4 EMs in series).
// Reference: IterativeClosestPointOptimizer.cpp:281-449 (the GN loop), :587-645 (correspondences).
#include "lo_pko_body.h"
#include "lo_solve.h"

namespace lo {

// LaRec / LaParams are declared in lo_device.h (the host allocates the buffers).

// Diagnostic build only (-DLO_PKO_STAMPS): chain 0 stores s_memtime at its stage boundaries into the context's
// DevState::dbg[8..15] (the main workgroup 0's PKO phases use dbg[0..6]).
#ifdef LO_PKO_STAMPS
#define LA_STAMP(c, i) do { if ((c) == 0 && threadIdx.x == 0) L.stamp[i] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define LA_STAMP(c, i) do { } while (0)
#endif

// Normal-equation partials of one GN iteration over the scan's 256-point blocks, NW/4 blocks per pass, into LDS:
// each block's partial is formed exactly as acc_candidate / accumulate_body form it (one point per thread, fp32
// wave totals, fp64 sum over the block's 4 waves in wave order).
template <int NW>
__device__ __forceinline__ void la_accumulate(const KParams& P, const int32_t* slot, const float (&T)[12],
                                              double scale, float dl, double* s_part) {
    constexpr int kG = NW / kWavesPerBlock;
    __shared__ float s_acc[NW][kNE];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int n = scan_n(P), nb = P.nb_acc;
    for (int vb0 = 0; vb0 < nb; vb0 += kG) {
        const int vb = vb0 + wid / kWavesPerBlock;
        const int i = vb * kBlock + (wid % kWavesPerBlock) * kWave + lane;
        float acc[kNE];
#pragma unroll
        for (int k = 0; k < kNE; ++k) acc[k] = 0.0f;
        if (vb < nb && i < n) acc_point(P, slot, T, scale, dl, i, acc);
        wave_totals_f32<kNE>(acc, s_acc[wid]);
        __syncthreads();
        if (tid < kG * kNE) {
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
}

// find_correspondences (:587-645) at pose T into B.slot / B.wmask / B.blk_cnt, NW/4 blocks per pass: the slot,
// ballot and count of every block exactly as correspond_tail + corr_epilogue write them (no iteration-0 stats).
template <int NW>
__device__ __forceinline__ void la_correspond(const KParams& P, const ScanBufs& B, const float (&T)[12]) {
    constexpr int kG = NW / kWavesPerBlock;
    __shared__ int s_cnt[NW];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int n = scan_n(P), nb = P.nb;
    for (int vb0 = 0; vb0 < nb; vb0 += kG) {
        const int vb = vb0 + wid / kWavesPerBlock;
        const int i = vb * kBlock + (wid % kWavesPerBlock) * kWave + lane;
        int slot = -1;
        if (vb < nb && i < n) {
            float wx, wy, wz;
            transform_pt(T, P.pts[3 * i], P.pts[3 * i + 1], P.pts[3 * i + 2], wx, wy, wz);
            const int s = lookup_surfel(P.tab, P.log2cap, P.l1scale, wx, wy, wz);
            if (s >= 0) {
                const double r = residual_f64(P.tab[s], wx, wy, wz);
                if (!(r > P.maxd)) slot = s;            // the reference rejects only residual > max (NaN kept, :630)
            }
            B.slot[i] = slot;
        }
        const uint64_t m = __ballot(slot >= 0);
        if (lane == 0) {
            if (vb < nb) B.wmask[vb * kWavesPerBlock + wid % kWavesPerBlock] = m;
            s_cnt[wid] = __popcll(m);
        }
        __syncthreads();
        if (tid < kG && vb0 + tid < nb) {
            int c = 0;
#pragma unroll
            for (int w = 0; w < kWavesPerBlock; ++w) c += s_cnt[tid * kWavesPerBlock + w];
            B.blk_cnt[vb0 + tid] = c;
        }
        __syncthreads();
    }
}

// Candidate index of the selection (k_solve_pick's rule): alpha index bi > 0 -> candidate bi - 1, none -> NA.
__device__ __forceinline__ int la_candidate(const KParams& P, const double* js) {
    const int bi = pko_select_index(P, js);
    return bi > 0 ? bi - 1 : P.NA;
}
__device__ __forceinline__ double la_delta(const KParams& P, int c) { return c < P.NA ? P.alphas[c + 1] : P.min_scale; }

// Resolve the launch of iteration k - 2: c* from its main JS grid, its chain's record.  Every workgroup decides the
// same; with publish (one workgroup per launch) the record goes into DevState (logs, pose, iteration count, alpha,
// n_corr, status, done) as the one-iteration path leaves it.  Returns done; *c_out = c*.
__device__ int la_resolve(const KParams& P, const LaParams& L, int k, bool publish, int* c_out) {
    DevState* st = P.st;
    __shared__ int s_c, s_done;
    const int tid = threadIdx.x;
    if (tid < kWave) {
        const int par0 = ((k - 2) >> 1) & 1;
        const int done0 = st->done;                         // the previous main's INSUFFICIENT, or an earlier resolve
        const int c = la_candidate(P, L.jsM + static_cast<size_t>(par0) * (P.NA + 1));
        if (tid == 0) {
            const LaRec& R = L.rec[static_cast<size_t>(par0) * (P.NA + 1) + c];
            int done = done0;
            if (!done0) {
                const bool two = R.n_exec == 2;
                done = R.conv0 || !two || R.status1 != LO_OK || R.conv1 || k >= P.max_iters;
                if (publish) {
                    st->logs[k - 2] = R.log[0];
                    const lo_iter_log& last = (two && R.status1 == LO_OK) ? R.log[1] : R.log[0];
                    if (two && R.status1 == LO_OK) st->logs[k - 1] = R.log[1];
                    for (int q = 0; q < 12; ++q) st->pose[q] = last.pose[q];
                    st->iter = (two && R.status1 == LO_OK) ? k : k - 1;
                    st->alpha = last.alpha;
                    st->n_corr = two ? R.log[1].n_corr : R.log[0].n_corr;
                    if (two && R.status1 != LO_OK) st->status = R.status1;
                    if (done) st->done = 1;
                }
            }
            s_c = c;
            s_done = done;
        }
    }
    __syncthreads();
    *c_out = s_c;
    return s_done;
}

// One candidate's chain (see the file comment).  Bk: iteration k's correspondence buffers and pose.
template <int NW>
__device__ void la_chain(const KParams& P, const ScanBufs& Bk, const LaParams& L, int k, int c, int par,
                         int* s_pre) {
    const int tid = threadIdx.x;
    const size_t nc1 = static_cast<size_t>(P.NA) + 1;
    __shared__ double s_part[kFuseMaxBlocks * kNE];
    __shared__ double s_tot[kNE];
    __shared__ float s_pose[2][12];
    __shared__ int s_stop, s_n1;
    __shared__ double s_a1;
    LaRec* R = L.rec + static_cast<size_t>(par) * nc1 + c;

    // ---- iteration k with delta_c ----
    LA_STAMP(c, 0);
    int nc;
    double scale;
    pko_prefix<NW>(P, Bk, k, false, s_pre, nc, scale);
    if (nc < P.min_corr) return;                           // the main workgroups report INSUFFICIENT
    const double a0 = la_delta(P, c);
    float T[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) T[q] = Bk.pose_in[q];
    la_accumulate<NW>(P, Bk.slot, T, scale, static_cast<float>(a0), s_part);
    LA_STAMP(c, 1);
    solve_sums<kBlock>(s_part, P.nb_acc, s_tot);
    if (tid == 0) {
        lo_iter_log lg;
        const bool conv = solve_step(P, s_tot, T, s_pose[0], &lg);
        lg.n_corr = nc;
        lg.scale = scale;
        lg.alpha = a0;
        R->log[0] = lg;
        R->conv0 = conv ? 1 : 0;
        R->conv1 = 0;
        R->status1 = LO_OK;
        R->n_exec = 1;
        s_stop = (conv || k + 1 >= P.max_iters) ? 1 : 0;
    }
    __syncthreads();
    LA_STAMP(c, 2);
    if (s_stop) return;

    // ---- iteration k + 1: correspondences and the whole PKO on the chain's own buffers and GN state ----
    float T1[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) T1[q] = s_pose[0][q];
    ScanBufs Bx;
    Bx.res = nullptr;                                      // la_correspond stores no residuals
    Bx.slot = L.slotX + static_cast<size_t>(c) * L.n_cap;
    Bx.wmask = L.wmaskX + static_cast<size_t>(c) * (L.n_cap / kWave);
    Bx.blk_cnt = L.blkX + static_cast<size_t>(c) * kFuseMaxBlocks;
    Bx.js = L.jsC + static_cast<size_t>(c) * nc1;
    Bx.st = L.stC + c;
    Bx.pose_in = nullptr;
    la_correspond<NW>(P, Bx, T1);
    LA_STAMP(c, 3);
    if (tid < 12) Bx.st->pose[tid] = T1[tid];
    if (tid == 0) {
        Bx.st->scale = scale;
        Bx.st->done = 0;
        Bx.st->status = LO_OK;
        Bx.st->n_corr = 0;
    }
    __syncthreads();
    pko_body<NW, false>(P, Bx, k + 1, 0, 1);
    __syncthreads();
    LA_STAMP(c, 4);
#ifdef LO_PKO_STAMPS
    if (c == 0 && tid < 7) P.st->dbg[tid] = Bx.st->dbg[tid];    // chain 0's PKO phases replace the main's
#endif
    if (tid < kWave) {
        const int c1 = la_candidate(P, Bx.js);
        if (tid == 0) {
            s_n1 = Bx.st->n_corr;
            s_a1 = la_delta(P, c1);
            s_stop = Bx.st->status != LO_OK ? 1 : 0;
            if (s_stop) {                                     // iteration k + 1 found too few correspondences
                R->log[1].n_corr = s_n1;
                R->status1 = Bx.st->status;
                R->n_exec = 2;
            }
        }
    }
    __syncthreads();
    if (s_stop) return;
    const double a1 = s_a1;
    la_accumulate<NW>(P, Bx.slot, T1, scale, static_cast<float>(a1), s_part);
    LA_STAMP(c, 5);
    solve_sums<kBlock>(s_part, P.nb_acc, s_tot);
    if (tid == 0) {
        lo_iter_log lg;
        const bool conv = solve_step(P, s_tot, T1, s_pose[1], &lg);
        lg.n_corr = s_n1;
        lg.scale = scale;
        lg.alpha = a1;
        R->log[1] = lg;
        R->conv1 = conv ? 1 : 0;
        R->n_exec = 2;
        s_stop = (conv || k + 2 >= P.max_iters) ? 1 : 0;
    }
    __syncthreads();
    LA_STAMP(c, 6);
    if (s_stop) return;

    // ---- correspondences at pose_{k+2}: the next launch's iteration-(k+2) input if c is selected ----
    float T2[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) T2[q] = s_pose[1][q];
    const size_t set = static_cast<size_t>(par) * nc1 + c;
    ScanBufs Bo = Bx;
    Bo.slot = L.slotO + set * L.n_cap;
    Bo.wmask = L.wmaskO + set * (L.n_cap / kWave);
    Bo.blk_cnt = L.blkO + set * kFuseMaxBlocks;
    la_correspond<NW>(P, Bo, T2);
    LA_STAMP(c, 7);
}

// grid = G main workgroups + NA + 1 chains; k even.  Launch k reads the correspondences that k_correspond (k = 0) or
// the selected chain of launch k - 2 wrote, and writes the parity-(k/2 & 1) half of the double-buffered outputs.
__global__ __launch_bounds__(kLaThreads) void k_la(const KParams* __restrict__ Pp, LaParams L, int k, int G) {
    constexpr int NW = kLaThreads / kWave;
    const KParams& P = *Pp;                                // the scan's k_correspond stashed them (fields on demand)
    extern __shared__ int s_pre[];
    const int wg = blockIdx.x;
    const int par = (k >> 1) & 1;
    ScanBufs Bk = own_bufs(P);
    Bk.pose_in = P.st->pose;                               // k = 0: the initial pose (k_correspond's reset)
    if (k > 0) {
        int cs;
        if (la_resolve(P, L, k, wg == 0, &cs)) return;
        const size_t set = static_cast<size_t>(par ^ 1) * (P.NA + 1) + cs;
        Bk.slot = L.slotO + set * L.n_cap;
        Bk.wmask = L.wmaskO + set * (L.n_cap / kWave);
        Bk.blk_cnt = L.blkO + set * kFuseMaxBlocks;
        Bk.pose_in = L.rec[set].log[1].pose;               // the pose after iteration k - 1
        Bk.res = nullptr;                                  // a chain's correspondences: no stored residuals
    } else if (P.st->done) {
        return;
    }
    if (wg < G) {
        Bk.js = L.jsM + static_cast<size_t>(par) * (P.NA + 1);
        pko_body<NW, false>(P, Bk, k, wg, G);
        return;
    }
    la_chain<NW>(P, Bk, L, k, wg - G, par, s_pre);
}

// After the last lookahead launch: publish the selected chain of launch k_next - 2.
__global__ void k_la_finish(const KParams* __restrict__ Pp, LaParams L, int k_next) {
    const KParams& P = *Pp;
    int cs;
    la_resolve(P, L, k_next, true, &cs);
}

}  // namespace lo
