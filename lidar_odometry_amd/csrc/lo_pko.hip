// lo_pko.hip — the PKO kernels (k_pko_t single scan, k_pko_tb batched, k_pko_finish); the device code lives in
// lo_pko_body.h.
#include "lo_pko_body.h"

namespace lo {

template <int NW>
__global__ __launch_bounds__(NW * 64) void k_pko_t(KParams P, int it, int G) {
    pko_body<NW, false>(P, own_bufs(P), it, blockIdx.x, G);
}
// Reference-exact mode (lo_set_exact): the same launch with acc_candidate_exact as the candidates.
__global__ __launch_bounds__(256) void k_pko_tx(KParams P, int it, int G) {
    pko_body<4, false, true>(P, own_bufs(P), it, blockIdx.x, G);
}

// Batched launch: blockIdx.y = job, gridDim.x workgroups per job split its alpha grid.  <4, false>: the
// single-scan workgroup (few jobs); <1, true>: one wave per job that fits the GMM alone (many jobs: the
// launch is bound by fp64 issue, and single-wave workgroups spread over the SIMDs evenly).
template <int NW, bool ONE_WAVE>
__global__ __launch_bounds__(NW * 64) void k_pko_tb(const KParams* __restrict__ PB, int it) {
    const KParams& P = PB[blockIdx.y];
    pko_body<NW, ONE_WAVE>(P, own_bufs(P), it, blockIdx.x, gridDim.x);
}

template __global__ void k_pko_t<4>(KParams, int, int);
template __global__ void k_pko_tb<4, false>(const KParams*, int);
template __global__ void k_pko_tb<1, true>(const KParams*, int);

// PKO-only entry point: argmin of the JS grid -> DevState::alpha (lo_pko_scale_factor).
__global__ void k_pko_finish(KParams P) {
    DevState* st = P.st;
    const double a = pko_select_alpha(P);
    if (threadIdx.x == 0) st->alpha = a;
}

}  // namespace lo

namespace lo {

// Batched reference-exact GN step (lo_batch_* over reference-exact contexts, lockstep): one 256-thread workgroup per
// job: the JS-selected Huber delta's 43 sequential fp32 sums in correspondence order (exact_sums_wg, the speculative
// candidates' own code), the reference's fp32 LDLT and re-projected update, the job's state and log -- what the single
// scan's candidate + pick (or k_exact_terms + k_exact_solve) write for the same iteration, so the same bits.
__global__ __launch_bounds__(256) void k_exact_acc_b(const KParams* __restrict__ PB, int it) {
    const KParams& P = PB[blockIdx.x];
    DevState* st = P.st;
    if (st->done) return;
    extern __shared__ __attribute__((aligned(16))) float s_dyn[];   // kXcLdsBytes (16-B aligned: ds_read_b128)
    float* s_tot = s_dyn + kXcTotOff;
    __shared__ double s_alpha;
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid < kWave) {
        const double a = P.use_pko ? pko_select_alpha(P) : P.robust_delta;
        if (lane == 0) s_alpha = a;
    }
    __syncthreads();
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = st->pose[k];
    exact_sums_wg(P, T, st->scale, static_cast<float>(s_alpha), s_dyn, s_tot);
    if (tid != 0) return;
    float tf[kExactTerms], pn[12], delta[6];
    for (int k = 0; k < kExactTerms; ++k) tf[k] = s_tot[k];
    const bool conv = exact_solve_step(tf, T, P.tol_t, P.tol_r, pn, delta);
    st->alpha = s_alpha;
    for (int q = 0; q < 12; ++q) st->pose[q] = pn[q];
    if (it < LO_MAX_ITERS) {
        lo_iter_log& L = st->logs[it];
        for (int q = 0; q < 12; ++q) L.pose[q] = pn[q];
        L.n_corr = st->n_corr;
        L.scale = st->scale;
        L.alpha = s_alpha;
        L.cost = tf[42];
        int k = 0;
        for (int r = 0; r < 6; ++r) for (int c = r; c < 6; ++c) L.H[k++] = tf[r * 6 + c];
        for (int j = 0; j < 6; ++j) { L.g[j] = tf[36 + j]; L.delta[j] = delta[j]; }
    }
    st->iter = it + 1;
    if (conv) st->done = 1;
}

}  // namespace lo
