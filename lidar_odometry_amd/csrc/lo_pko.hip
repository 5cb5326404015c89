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
