// lo_icp.hip — host side of the C ABI declared in include/lo_icp.h.
//
// Owns one HIP stream per context, the device-resident surfel hash table, scan buffers, the PKO tables
// and the DevState that carries the Gauss-Newton loop.  lo_icp_optimize enqueues the whole loop
// (4 kernels x max_iterations) with no host synchronisation in between; the kernels read
// DevState::done and fall through once the scan has converged or failed.
#include <hipcub/hipcub.hpp>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "lo_ctx_internal.h"
#include "lo_device.h"
#include "lo_exact.h"
#include "lo_kdorder.h"
#include "lo_math.h"
#include "lo_pko_tables.h"
#include "lo_seqsum.h"
#include "lo_vfilter.h"

namespace lo {
__global__ void k_correspond(KParams P, int with_stats);
template <int NW> __global__ void k_pko_t(KParams P, int it, int G);
__global__ void k_pko_tx(KParams P, int it, int G);
__global__ void k_pko_finish(KParams P);
__global__ void k_accumulate(KParams P, int it, int fuse);
__global__ void k_solve(KParams P, int it, int ne_only);
__global__ void k_solve_pick(KParams P, int it);
__global__ void k_solve_correspond(KParams P, int it);
__global__ void k_solve_knn(KParams P, int it);
__global__ void k_pick_knn(KParams P, int it);
__global__ void k_pick_correspond(KParams P, int it);
__global__ void k_pick(KParams P, int it);
struct Pose12 { float v[12]; };
__global__ void k_init(DevState* st, Pose12 T, double scale, double alpha);
__global__ void k_export_pose(const DevState* st, float* out);
__global__ void k_wait_seq(uint32_t* fin, uint32_t seq, DevState* st, uint32_t* hbroken, unsigned long long bound);
__global__ void k_wait_final(uint32_t* fin, uint32_t seq, DevState* st, uint32_t* hbroken, unsigned long long bound);
__global__ void k_knn(KParams P);
__global__ void k_knn_brute(KParams P);
__global__ void k_knn_brute_w(KParams P);
__global__ void k_knn_all(KParams P);
__global__ void k_pick_knn_all(KParams P, int it);
__global__ void k_inlier_all(KParams P);
__global__ void k_knn_reset(KParams P);
__global__ void k_plane(KParams P, int with_stats);
__global__ void k_inlier(KParams P);
__global__ void k_correspond_b(const KParams* PB, int with_stats, int init);
template <int NW, bool ONE_WAVE> __global__ void k_pko_tb(const KParams* PB, int it);
__global__ void k_accumulate_b(const KParams* PB, int it);
template <bool SOLVE> __global__ void k_accumulate_b1(const KParams* PB, int it);
__global__ void k_solve_b1(const KParams* PB, int it);
__global__ void k_solve_b(const KParams* PB, int it);
__global__ void k_export_batch(const KParams* PB, lo_batch_rec* out);
__global__ void k_exact_acc_b(const KParams* PB, int it);
void launch_exact_scale_cb(const KParams* PB, int njobs, int n_max, hipStream_t s);
struct MapPatchRec;
__global__ void k_map_patch(Slot* tab, uint32_t log2cap, const MapPatchRec* rec, int n);
struct FitJob {
    uint64_t key;
    int32_t off, m;
};
struct FitOut;
__global__ void k_surfel_fit(const FitJob* jobs, const float* cs, int n, float thr, Slot* tab, uint32_t log2cap,
                             FitOut* out);
void launch_exact_scale(const KParams& P, int n, double* sorted, hipStream_t s);
hipError_t exact_scale_rank_prepare();
hipError_t exact_scale_m_prepare();
hipError_t exact_scale_c_prepare();
void launch_exact_scale_c(const KParams& P, hipStream_t s);
void launch_exact_scale_m(const KParams& P, const uint64_t* runs, uint64_t* sorted, hipStream_t s);
void launch_seq_sum_diag(const double* x, int n, double* sort, double* out, long long* stats, hipStream_t s);
void launch_mw_sums(const float* col0, int ld, int ncol, int n_cap, const int* n_dev, const DevState* st, const MwBuf& B,
                    float* out, long long* stats, hipStream_t s, bool factored);
size_t mw_bytes(int ncol, int n_cap);
MwBuf mw_layout(void* mem, int ncol, int n_cap);
hipError_t mw_clear(const MwBuf& B, int ncol, hipStream_t s);
#ifndef LO_EXACT_FACTORED
#define LO_EXACT_FACTORED 1                                  // lo_exact.h kExactFactored
#endif
void launch_mwm_scale(KParams P, const double* sorted, const MwmBuf& B, hipStream_t s);
size_t mwm_bytes(int n_cap);
MwmBuf mwm_layout(void* mem, int n_cap);
__global__ void k_exact_resid(KParams P, double* out);
__global__ void k_exact_terms(KParams P);
__global__ void k_exact_solve(KParams P, int it);
__global__ void k_exact_finish(KParams P, int it);
}  // namespace lo

using namespace lo;

// Dense uniform grid over a point set (the kd-tree's role): points sorted by cell, x fastest, index order
// inside a cell; start[cell] = first point, start[ncell] = m.
struct PointGrid {
    float4* d_pts = nullptr;
    size_t pts_cap = 0;
    uint32_t* d_start = nullptr;
    size_t start_cap = 0;
    uint32_t* d_vpos = nullptr;     // nanoflann visit order (lo_kdorder.h): vAcc_ position per original index
    size_t vpos_cap = 0;
    KdNode* d_nodes = nullptr;      //   and the tree's nodes (root = 0)
    size_t nodes_cap = 0;
    bool has_order = false;         // d_vpos / d_nodes hold the visit order of the current points
    bool all = false;               // d_pts in index order, no cells (all_pairs_upload: k_knn_all / k_inlier_all)
    void* h_stage = nullptr;        // pinned upload staging (grid_build)
    size_t stage_cap = 0;
    int m = 0;
    int org[3] = {0, 0, 0}, dim[3] = {1, 1, 1};
    float h = 1.0f;
};

// ctx_grid_from_device's scratch: the bounds readback, keys / values (and their sorted copies), cell counts, hipCUB temp
struct DevGridScratch {
    float* d_bounds = nullptr;
    float* h_bounds = nullptr;
    uint32_t* d_keys = nullptr;
    size_t keys_cap = 0;
    uint32_t* d_counts = nullptr;
    size_t counts_cap = 0;
    unsigned char* d_tmp = nullptr;
    size_t tmp_cap = 0;
};

struct lo_ctx {
    lo_config cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = true;
    std::string err;
    // scan buffers
    float* d_pts = nullptr;
    int32_t* d_slot = nullptr;
    double* d_res_pko = nullptr;    // per-point residual of the accepted correspondences (the PKO sample reads it)
    uint64_t* d_wmask = nullptr;
    int32_t* d_blk_cnt = nullptr;
    double* d_blk_sum = nullptr;
    double* d_blk_m2 = nullptr;
    double* d_blk_part = nullptr;
    double* d_acc_part = nullptr;   // speculative normal equations (allocated on the first PKO optimize)
    float* d_cand_rec = nullptr;    //   and each candidate's solved GN step [NA + 1][kCandWords]
    unsigned* d_cand_cnt = nullptr; //   per-candidate workgroup arrivals (zero between launches)
    bool presolve = true;           //   candidates solve inside the PKO launch (LO_PRESOLVE=0: k_solve_* instead)
    bool exact = true;              // lo_set_exact: the reference's own arithmetic order (lo_exact.hip) -- the default;
                                    //   lo_set_exact(ctx, 0) opts into the fast mode (fp64 tree sums, not parity-safe)
    uint64_t cfg_gen = 0;           // bumped by lo_update_config and by (re)allocations of the PKO / candidate buffers: a
                                    //   batch's cached device KParams of this context are stale once it changes
    float* d_ex_terms = nullptr;
    size_t ex_cap = 0;              //   floats in d_ex_terms
    float* d_ex_tot = nullptr;      //   large scans: the 43 sums (launch_mw_sums -> k_exact_finish)
    double* d_ex_rank = nullptr;    //   the iteration-0 residuals in sorted order (k_rank_sort, kExactMaxPoints), or
                                    //   up to kExactMergeMax points: the correspondence blocks' sorted runs
    bool ex_merge = false;          //   this scan's exact scale runs in one launch (k_exact_scale_c: counting sort + sums)
    bool ex_merge_presort = false;  //   ... or from the correspondence blocks' presorted runs (LO_EXACT_PRESORT, A/B)
    bool ex_attr = false;           //   the exact-scale kernels' dynamic-LDS attributes are set (per context)
    void* d_mw = nullptr;           //   large scans: head records of the 43 column sums (lo_seqsum.h MwBuf)
    size_t mw_n_cap = 0;            //   the scan size d_mw is laid out for
    MwBuf mw{};
    void* d_mwm = nullptr;          //   large scans: head records of the iteration-0 scale's two sums (MwmBuf)
    MwmBuf mwm{};
    double* d_ex_res = nullptr;     //   scans beyond kExactMaxPoints: residuals, sorted residuals, hipCUB scratch
    double* d_ex_sorted = nullptr;
    void* d_ex_sort_tmp = nullptr;
    size_t ex_res_cap = 0, ex_sort_tmp_bytes = 0;
    double* d_js = nullptr;
    double* d_res = nullptr;        // parity entry points (per-point residual / direct residual input)
    size_t res_cap = 0;
    uint8_t* d_u8 = nullptr;
    DevState* d_st = nullptr;
    DevState* h_st = nullptr;       // pinned
    int* h_nf = nullptr;            // pinned: the device-filtered scan's count, read back with the result
    bool nf_valid = false;          //   h_nf holds the last device-filtered scan's count (lo_icp_result)
    // map
    Slot* d_tab = nullptr;
    size_t tab_cap = 0;             // allocated slots
    uint32_t log2cap = 1;
    size_t n_surfels = 0;
    // in-place table patches (lo_map_patch_surfels): the keys resident on the device, tombstones left by erases,
    // a pinned staging buffer + device copy of the patch records, and the synced host map (lo_map_sync_voxelmap)
    std::unordered_set<uint64_t> resident;
    size_t n_tomb = 0;
    void* h_patch = nullptr;
    void* d_patch = nullptr;
    size_t patch_cap = 0;
    hipEvent_t ev_patch = nullptr;
    uint64_t map_src = 0, map_epoch = 0, map_pos = 0;
    uint64_t tab_gen = 0;           // bumped by every full upload (a pending fit's results no longer apply to it)
    uint64_t tab_edit = 0;          // bumped by every change of the table (uploads, patches, fits, a device map's claim)
    // lo_map_sync_surfels: the surfel set last synced through it (key -> normal, centroid), valid while the table has
    // not been changed by anything else since (mirror_edit == tab_edit)
    std::unordered_map<uint64_t, std::array<float, 6>> smirror;
    uint64_t mirror_edit = ~0ull;
    uint64_t devmap_gen = 0;        // the generation a device map (lo_devmap) reserved and maintains
    // deferred surfel fits of a synced host map (lo::ctx_fit_surfels): pinned in / out staging, device copies
    void* h_fit_in = nullptr;
    void* d_fit_in = nullptr;
    size_t fit_in_cap = 0;
    FitResult* h_fit_out = nullptr;
    FitResult* d_fit_out = nullptr;
    size_t fit_out_cap = 0;
    hipEvent_t ev_fit = nullptr;
    uint64_t fit_ticket = 0;        // the launch whose results sit in h_fit_out (0: none)
    uint64_t fit_gen = 0;           //   and the table generation it patched
    std::vector<uint64_t> fit_keys; //   its packed keys, job order
    bool fit_reconciled = false;    //   its planarity failures already removed from `resident`
    float fit_thr = 0.0f;
    // KDTree variant: dense grid over the L0 centroids + per-point neighbour / plane / residual buffers
    bool kd = false;
    PointGrid grid;                 // the map's L0 centroids (lo_map_set_points, or ctx_grid_from_device)
    DevGridScratch gscr;
    bool grid_dev = false;          // the grid was built on the device (no kd visit order; ties re-run, lo_icp_result)
    int kd_reruns = 0;              //   scans re-run with the order after such a tie (lo_kd_reruns)
    PointGrid lgrid;                // loop closure: the matched keyframe's local map (lo_icp_optimize_loop)
    uint64_t loop_reruns = 0;       //   solves rerun with the kd visit order (a deciding distance tie)
    int32_t* d_kd_nbr = nullptr;
    int32_t* d_kd_unres = nullptr;
    double* d_kd_res = nullptr;
    Slot* d_kd_plane = nullptr;
    // device preprocessing (FastVoxelFilter): raw staging for host input + filter work buffers
    float* d_raw = nullptr;
    size_t raw_cap = 0;
    VfBuffers vf;
    bool last_dev_count = false;    // last optimize took its point count from the device filter
    // PKO tables
    PkoTables tables;
    double* d_alphas = nullptr;
    double* d_Z = nullptr;
    int32_t* d_tabs_i = nullptr;    // small_off | small_perm | base | ev_off | ev_steps | km_draws
    size_t off_small_off = 0, off_small_perm = 0, off_base = 0, off_ev_off = 0, off_ev_steps = 0, off_km = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // in-step timing of each scan's first correspondence launch (lo_set_stage_timing / lo_stage_time)
    bool stage_timing = false;
    std::vector<hipEvent_t> st_ev;  // pairs: [2 i] before, [2 i + 1] after
    int st_n = 0;
    unsigned long long* d_span = nullptr;   // in-kernel span stamps (kSpanWords per launch): stage-timed launch i at
                                            //   kSpanWords i; lo_bench_kernel 5 at kSpanWords kStageEvents
    float T_init[12];
    size_t last_n = 0;
    bool pending = false;
    // scan pipeline (lo_set_pipeline; on by default): GN iterations >= pipe_main of a small PKO scan go to a tail
    // stream, and the context stream is held (k_wait_final) only until the scan's result is final -- a converged
    // scan's early-exit launches drain beside the next scan instead of in front of it.  The tail starts when the main
    // part is done (k_wait_seq polls the word the main part's last pick sets); no HIP events on the hot path (every
    // marker packet costs ~5-7 us of device time between two kernels).
    bool pipe = true;
    int pipe_main = 2;
    int pko_groups = 0;             // EM workgroups per PKO launch (lo_set_pko_groups / LO_PKO_GROUPS; 0 = one per alpha)
    bool pko_solo = false;          // LO_PKO_SOLO=1 (A/B): the speculative PKO launch asks for enough LDS that one
                                    //   workgroup holds a CU alone (no other launch's waves on its SIMDs)
    hipStream_t s_tail = nullptr;
    uint32_t pipe_seq = 0;
    uint32_t* d_fin = nullptr;      // [0] the last scan whose result is final (publish_final), [1] main part done,
                                    // [2] signal_main's block count, [3] broken (a wait timed out; sticky)
    uint32_t* h_broken = nullptr;   // pinned, device-mapped: the seq of the scan whose wait timed out (0: none)
    uint32_t* d_hbroken = nullptr;
    unsigned long long pipe_bound = 200000000ull;   // wait bound in 100 MHz ticks (2 s; LO_PIPE_WAIT_MS)
    uint32_t pipe_fail_at = 0;      // test hook (LO_PIPE_FAIL_AT=k): the k-th pipelined scan's tail wait gives up at once
    unsigned pipe_timeouts = 0;     // times a wait timed out and the pipeline was switched off (lo_pipeline_status)
    unsigned pipe_reruns = 0;       // synchronous scans re-run on one stream after such a timeout
    const float* last_pts = nullptr;   // the scan in flight (a re-run after a pipeline timeout)
    const int* last_ndev = nullptr;
    bool sync_call = false;         // the optimize in flight is a synchronous call: HIP events time it (gpu_ms)
    bool last_timed = false;
};

#define LO_HIP(ctx, call)                                                                  \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) {                                                            \
            (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);               \
            return LO_ERR_HIP;                                                             \
        }                                                                                  \
    } while (0)

// PKO workgroups: one alpha of the JS grid per workgroup (each fits the GMM redundantly), capped at kPkoMaxWGs
static int pko_grid(const lo_config& g) { return std::max(1, std::min(kPkoMaxWGs, g.num_alpha_segments)); }
// the context's EM workgroup count: pko_groups (lo_set_pko_groups; 0 = one alpha per workgroup, pko_grid)
static int pko_grid(const lo_ctx* c) {
    const int full = pko_grid(c->cfg);
    return c->pko_groups > 0 ? std::min(full, c->pko_groups) : full;
}

static void launch_pko(lo_ctx* c, const KParams& P, int it) {
    // dynamic LDS for the per-block prefix (nb ints; 64 KB only at the 4M-point maximum)
    const size_t pre_bytes = static_cast<size_t>(std::max(P.nb, 1)) * sizeof(int);
    // 4 waves: the EM runs one GMM component per wave (gmm_fit_split), up to 256 samples (4 per lane)
    const int G = pko_grid(c);
    hipLaunchKernelGGL(k_pko_t<4>, dim3(G), dim3(256), pre_bytes, c->stream, P, it, G);
}

// Small scans with PKO: the PKO launch also evaluates the normal equations for every alpha candidate
// (acc_candidate, lo_pko.hip, (NA + 1) x ceil(nb_acc / kSpecBlocksPerWG) extra workgroups); k_solve_pick then
// solves the selected one.
static bool spec_ok(const KParams& P) { return P.use_pko && P.acc_part && P.nb_acc <= kFuseMaxBlocks; }

constexpr size_t kPkoSoloBytes = 64 * 1024;   // + the ~22-27 KB static part: more than half of a CU's 160 KB
static void launch_pko_spec(lo_ctx* c, const KParams& P, int it, hipStream_t s = nullptr) {
    size_t pre_bytes = static_cast<size_t>(std::max(P.nb, 1)) * sizeof(int);
    const int G = pko_grid(c);
    int W = (P.nb_acc + kSpecBlocksPerWG - 1) / kSpecBlocksPerWG;
    if (P.exact_cand) {                                  // one workgroup per exact candidate, factor rows in LDS
        W = 1;
        pre_bytes = std::max(pre_bytes, kXcLdsBytes);
    }
    if (c->pko_solo) pre_bytes = std::max(pre_bytes, kPkoSoloBytes);
    if (P.exact_cand) hipLaunchKernelGGL(k_pko_tx, dim3(G + (P.NA + 1) * W), dim3(256), pre_bytes, s ? s : c->stream, P, it, G);
    else hipLaunchKernelGGL(k_pko_t<4>, dim3(G + (P.NA + 1) * W), dim3(256), pre_bytes, s ? s : c->stream, P, it, G);
}

// One GN iteration after the correspondence stage: PKO with the speculative normal equations + k_solve_pick
// (small scans), else PKO, then k_accumulate whose last block solves (small) or k_solve over 1024 threads (large).
static void launch_gn_tail(lo_ctx* c, const KParams& P, int it) {
    const dim3 blk(kBlock);
    if (spec_ok(P)) {
        launch_pko_spec(c, P, it);
        hipLaunchKernelGGL(k_solve_pick, dim3(1), blk, 0, c->stream, P, it);
        return;
    }
    launch_pko(c, P, it);
    if (P.nb_acc <= kFuseMaxBlocks) {
        hipLaunchKernelGGL(k_accumulate, dim3(P.nb_acc), blk, 0, c->stream, P, it, 1);
    } else {
        hipLaunchKernelGGL(k_accumulate, dim3(P.nb_acc), blk, 0, c->stream, P, it, 0);
        hipLaunchKernelGGL(k_solve, dim3(1), dim3(kSolveThreads), 0, c->stream, P, it, 0);
    }
}

static int ensure_acc_part(lo_ctx* c) {
    if (c->d_acc_part || !c->cfg.use_adaptive_m_estimator) return LO_OK;
    const size_t cand = static_cast<size_t>(c->cfg.num_alpha_segments) + 1;
    LO_HIP(c, hipMalloc(&c->d_acc_part, cand * kFuseMaxBlocks * kNE * sizeof(double)));
    LO_HIP(c, hipMalloc(&c->d_cand_rec, cand * kCandWords * sizeof(float)));
    LO_HIP(c, hipMalloc(&c->d_cand_cnt, cand * sizeof(unsigned)));
    LO_HIP(c, hipMemset(c->d_cand_cnt, 0, cand * sizeof(unsigned)));
    ++c->cfg_gen;
    // the exact candidates' staging sits in the PKO launch's dynamic LDS (beyond the 64 KB default with the static part)
    LO_HIP(c, hipFuncSetAttribute(reinterpret_cast<const void*>(k_pko_tx), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(std::max(kXcLdsBytes + 16384, kPkoSoloBytes))));
    LO_HIP(c, hipFuncSetAttribute(reinterpret_cast<const void*>(k_pko_t<4>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(kPkoSoloBytes)));
    return LO_OK;
}

// Scan pipeline (first pipelined scan): the tail stream and the two flag words.
static int pipe_alloc(lo_ctx* c) {
    if (c->d_fin) return LO_OK;
    LO_HIP(c, hipStreamCreateWithFlags(&c->s_tail, hipStreamNonBlocking));
    LO_HIP(c, hipMalloc(&c->d_fin, 4 * sizeof(uint32_t)));
    LO_HIP(c, hipMemset(c->d_fin, 0, 4 * sizeof(uint32_t)));
    LO_HIP(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_broken), sizeof(uint32_t),
                            hipHostMallocMapped | hipHostMallocCoherent));
    *c->h_broken = 0;
    LO_HIP(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&c->d_hbroken), c->h_broken, 0));
    LO_HIP(c, hipDeviceSynchronize());              // zeroed before either stream's first poll
    return LO_OK;
}


// Both streams of the context drained (lo_sync, lo_set_stream, lo_destroy).
static hipError_t sync_all(lo_ctx* c) {
    hipError_t e = c->stream ? hipStreamSynchronize(c->stream) : hipSuccess;
    if (e == hipSuccess && c->s_tail) e = hipStreamSynchronize(c->s_tail);
    return e;
}

// A pipeline wait timed out (the dispatcher ran the two streams out of submission order): drain both streams, switch
// the pipeline off for this context, clear the flag words.  Scans enqueued before this point report LO_ERR_PIPELINE
// (their tails left without touching anything); a synchronous call re-runs its scan on one stream (lo_icp_result).
static int pipe_recover(lo_ctx* c) {
    LO_HIP(c, sync_all(c));
    c->pipe = false;
    ++c->pipe_timeouts;
    c->err = "scan pipeline: a device-side wait timed out (the two streams were not run concurrently, e.g. rocprofv3 "
             "counter collection); pipeline switched off for this context";
    LO_HIP(c, hipMemset(c->d_fin, 0, 4 * sizeof(uint32_t)));
    LO_HIP(c, hipStreamSynchronize(nullptr));
    __atomic_store_n(c->h_broken, 0u, __ATOMIC_RELEASE);
    return LO_OK;
}
static bool pipe_flagged(const lo_ctx* c) { return c->h_broken && __atomic_load_n(c->h_broken, __ATOMIC_ACQUIRE) != 0u; }

static void set_kd_params(lo_ctx* c, KParams& P, const PointGrid& G) {
    P.tab = c->d_kd_plane;
    P.kd_pts = G.d_pts;
    P.kd_start = G.d_start;
    P.kd_vpos = G.has_order ? G.d_vpos : nullptr;
    P.kd_nodes = G.has_order ? G.d_nodes : nullptr;
    P.kd_m = G.m;
    for (int a = 0; a < 3; ++a) { P.kd_org[a] = G.org[a]; P.kd_dim[a] = G.dim[a]; }
    P.kd_h = G.h;
    P.kd_all = G.all ? 1 : 0;
    P.kd_nbr = c->d_kd_nbr;
    P.kd_unres = c->d_kd_unres;
    P.kd_res = c->d_kd_res;
    P.kd_plane = c->d_kd_plane;
}

static KParams make_params(lo_ctx* c, const float* d_pts, int n) {
    KParams P{};
    const lo_config& g = c->cfg;
    P.pts = d_pts;
    P.n = n;
    P.nb = (n + kBlock - 1) / kBlock;
    P.nb_acc = P.nb < kAccBlocks ? (P.nb > 0 ? P.nb : 1) : kAccBlocks;
    P.tab = c->d_tab;
    P.log2cap = c->log2cap;
    P.l1scale = g.voxel_size * static_cast<float>(g.hierarchy_factor);   // PointToVoxelKey (VoxelMap.cpp:51-52)
    P.max_iters = g.max_iterations;
    P.tol_t = g.translation_tolerance;
    P.tol_r = g.rotation_tolerance;
    P.maxd = g.max_correspondence_distance;
    P.min_corr = g.min_correspondence_points;
    P.robust = g.use_robust_loss;
    P.robust_delta = g.robust_loss_delta;
    P.cauchy_loss = g.loss_cauchy;
    P.use_pko = g.use_adaptive_m_estimator;
    P.S = g.gmm_sample_size;
    P.K = g.gmm_components;
    P.NA = g.num_alpha_segments;
    P.pko_kernel = g.pko_kernel;
    P.min_scale = g.min_scale_factor;
    P.trunc = g.truncated_threshold;
    P.alphas = c->d_alphas;
    P.Z = c->d_Z;
    P.small_off = c->d_tabs_i + c->off_small_off;
    P.small_perm = c->d_tabs_i + c->off_small_perm;
    P.base = c->d_tabs_i + c->off_base;
    P.ev_off = c->d_tabs_i + c->off_ev_off;
    P.ev_steps = c->d_tabs_i + c->off_ev_steps;
    P.km_draws = c->d_tabs_i + c->off_km;
    P.slot = c->d_slot;
    P.wmask = c->d_wmask;
    P.blk_cnt = c->d_blk_cnt;
    P.blk_sum = c->d_blk_sum;
    P.blk_m2 = c->d_blk_m2;
    P.blk_part = c->d_blk_part;
    P.acc_part = c->d_acc_part;
    P.cand_rec = c->presolve ? c->d_cand_rec : nullptr;   // candidates pre-solve (k_pick*, KDTree: k_pick_knn)
    P.cand_cnt = c->d_cand_cnt;
    P.js = c->d_js;
    P.res_dbg = nullptr;
    P.res_out = c->d_res_pko;
    P.direct_res = nullptr;
    P.st = c->d_st;
    P.em_stat = c->stage_timing ? reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(c->d_st) +
                                                                        offsetof(DevState, em_stat))
                                : nullptr;                  // the lead PKO workgroup's EM clock (stage timing)
    if (c->kd) set_kd_params(c, P, c->grid);             // KDTree path: downstream kernels read per-point planes
    return P;
}

static int validate_config(const lo_config* g, std::string& err) {
    if (!g) { err = "null config"; return LO_ERR_ARG; }
    if (g->max_iterations < 1 || g->max_iterations > LO_MAX_ITERS) { err = "max_iterations out of [1, 64]"; return LO_ERR_ARG; }
    // >= 1: an iteration with no correspondence always fails (the reference would fall back to robust_loss_delta
    // with an empty system, IterativeClosestPointOptimizer.cpp:298-331; never reached with its default of 10)
    if (g->min_correspondence_points < 1) { err = "min_correspondence_points must be >= 1"; return LO_ERR_ARG; }
    if (g->gmm_sample_size < 1 || g->gmm_sample_size > kMaxS) { err = "gmm_sample_size out of [1, 256]"; return LO_ERR_ARG; }
    if (g->gmm_components < 1 || g->gmm_components > 3) { err = "gmm_components out of [1, 3]"; return LO_ERR_ARG; }
    if (g->pko_kernel < LO_PKO_HUBER || g->pko_kernel > LO_PKO_PSEUDO_HUBER) { err = "pko_kernel out of [0, 5]"; return LO_ERR_ARG; }
    if (g->num_alpha_segments < 1 || g->num_alpha_segments > kMaxAlpha) { err = "num_alpha_segments out of [1, 1000]"; return LO_ERR_ARG; }
    if (!(g->voxel_size > 0.0f)) { err = "voxel_size must be positive"; return LO_ERR_ARG; }   // VoxelMap.cpp:28-30
    if (g->hierarchy_factor <= 0 || g->hierarchy_factor % 2 == 0) { err = "hierarchy_factor must be positive and odd"; return LO_ERR_ARG; }
    if (g->max_points < 1 || g->max_points > kMaxBlocks * kBlock) { err = "max_points out of [1, 4194304]"; return LO_ERR_ARG; }
    return LO_OK;
}

extern "C" {

void lo_config_default_kitti(lo_config* c) {
    std::memset(c, 0, sizeof(*c));
    c->max_iterations = 4;
    c->translation_tolerance = 0.005;
    c->rotation_tolerance = 0.005;
    c->max_correspondence_distance = 1.0;
    c->min_correspondence_points = 10;
    c->use_robust_loss = 1;
    c->robust_loss_delta = 0.1;
    c->loss_cauchy = 0;
    c->use_adaptive_m_estimator = 1;
    c->min_scale_factor = 0.1;
    c->max_scale_factor = 10.0;
    c->num_alpha_segments = 100;
    c->truncated_threshold = 10.0;
    c->gmm_components = 3;
    c->gmm_sample_size = 100;
    c->pko_kernel = LO_PKO_HUBER;
    c->voxel_size = 0.5f;
    c->hierarchy_factor = 3;
    c->use_surfel_correspondence = 1;
    c->max_points = 1 << 17;
}

int lo_pko_kernel_from_name(const char* name) {
    if (!name) return LO_PKO_CAUCHY;
    const std::string k(name);
    if (k == "huber") return LO_PKO_HUBER;
    if (k == "cauchy") return LO_PKO_CAUCHY;
    if (k == "tukey") return LO_PKO_TUKEY;
    if (k == "welsch") return LO_PKO_WELSCH;
    if (k == "gemanMcClure") return LO_PKO_GEMAN_MCCLURE;
    if (k == "pseudoHuber") return LO_PKO_PSEUDO_HUBER;
    return LO_PKO_CAUCHY;                                  // "Default to Cauchy" (AdaptiveMEstimator.cpp:150-155)
}

void lo_config_default_mid360(lo_config* c) {
    lo_config_default_kitti(c);
    c->voxel_size = 0.4f;   // config/mid360.yaml:19
}

const char* lo_last_error(const lo_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }
int lo_get_config(const lo_ctx* ctx, lo_config* out) {
    if (!ctx || !out) return LO_ERR_ARG;
    *out = ctx->cfg;
    return LO_OK;
}
int lo_device(const lo_ctx* ctx) { return ctx ? ctx->device : -1; }
void* lo_stream(lo_ctx* ctx) { return ctx ? static_cast<void*>(ctx->stream) : nullptr; }

// per-point buffers of the KDTree correspondence stage (KDTree map mode, and the loop-closure ICP of any context)
static int kd_alloc(lo_ctx* c) {
    if (c->d_kd_nbr) return LO_OK;
    const size_t NB = (static_cast<size_t>(c->cfg.max_points) + kBlock - 1) / kBlock;
    LO_HIP(c, hipMalloc(&c->d_kd_nbr, NB * kBlock * 5 * sizeof(int32_t)));
    LO_HIP(c, hipMalloc(&c->d_kd_unres, NB * kBlock * sizeof(int32_t)));
    LO_HIP(c, hipMalloc(&c->d_kd_res, NB * kBlock * sizeof(double)));
    LO_HIP(c, hipMalloc(&c->d_kd_plane, NB * kBlock * sizeof(Slot)));
    for (const void* f : {reinterpret_cast<const void*>(&k_knn_all), reinterpret_cast<const void*>(&k_pick_knn_all),
                          reinterpret_cast<const void*>(&k_inlier_all)})
        LO_HIP(c, hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kKnnAllMax * sizeof(float4)));
    for (PointGrid* G : {&c->grid, &c->lgrid}) {          // empty grid until a point set is uploaded
        LO_HIP(c, hipMalloc(&G->d_start, 2 * sizeof(uint32_t)));
        LO_HIP(c, hipMemset(G->d_start, 0, 2 * sizeof(uint32_t)));
        G->start_cap = 2;
        G->h = 2.0f * c->cfg.voxel_size;
    }
    return LO_OK;
}

// PKO tables (alpha grid, Z(alpha), the shuffle tables, the k-means draws), host-built for the context's config
// Built for config g into new buffers first; the context's tables and pointers change only once everything succeeded
// (a failed update leaves the old ones in place).
static int upload_pko_tables(lo_ctx* c, const lo_config& g) {
    PkoTables t;
    build_pko_tables(t, g.gmm_sample_size, g.gmm_components, g.max_points, g.min_scale_factor,
                     g.max_scale_factor, g.num_alpha_segments, g.truncated_threshold, g.pko_kernel);
    std::vector<int32_t> all;
    size_t off[6];
    auto append = [&](const std::vector<int32_t>& v, size_t& o) { o = all.size(); all.insert(all.end(), v.begin(), v.end()); all.push_back(0); };
    append(t.small_off, off[0]);
    append(t.small_perm, off[1]);
    append(t.base, off[2]);
    append(t.ev_off, off[3]);
    append(t.ev_steps, off[4]);
    append(t.km_draws, off[5]);
    double *a = nullptr, *z = nullptr;
    int32_t* ti = nullptr;
    auto fail = [&](hipError_t e, const char* what) {
        for (void* p : {static_cast<void*>(a), static_cast<void*>(z), static_cast<void*>(ti)}) if (p) (void)hipFree(p);
        c->err = std::string(what) + ": " + hipGetErrorString(e);
        return LO_ERR_HIP;
    };
    hipError_t e;
    if ((e = hipMalloc(&a, t.alphas.size() * sizeof(double))) != hipSuccess) return fail(e, "hipMalloc alphas");
    if ((e = hipMalloc(&z, t.Z.size() * sizeof(double))) != hipSuccess) return fail(e, "hipMalloc Z");
    if ((e = hipMalloc(&ti, all.size() * sizeof(int32_t))) != hipSuccess) return fail(e, "hipMalloc tables");
    if ((e = hipMemcpy(a, t.alphas.data(), t.alphas.size() * sizeof(double), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(z, t.Z.data(), t.Z.size() * sizeof(double), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(ti, all.data(), all.size() * sizeof(int32_t), hipMemcpyHostToDevice)) != hipSuccess)
        return fail(e, "hipMemcpy PKO tables");
    for (void* p : {static_cast<void*>(c->d_alphas), static_cast<void*>(c->d_Z), static_cast<void*>(c->d_tabs_i)})
        if (p) (void)hipFree(p);
    c->d_alphas = a;
    c->d_Z = z;
    c->d_tabs_i = ti;
    c->off_small_off = off[0]; c->off_small_perm = off[1]; c->off_base = off[2];
    c->off_ev_off = off[3]; c->off_ev_steps = off[4]; c->off_km = off[5];
    c->tables = std::move(t);
    ++c->cfg_gen;
    return LO_OK;
}

static int ctx_alloc(lo_ctx* c) {
    const lo_config& g = c->cfg;
    LO_HIP(c, hipSetDevice(c->device));
    LO_HIP(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    const size_t N = static_cast<size_t>(g.max_points);
    const size_t NB = (N + kBlock - 1) / kBlock;
    LO_HIP(c, hipMalloc(&c->d_pts, N * 3 * sizeof(float)));
    LO_HIP(c, hipMalloc(&c->d_slot, NB * kBlock * sizeof(int32_t)));
    LO_HIP(c, hipMalloc(&c->d_res_pko, NB * kBlock * sizeof(double)));
    LO_HIP(c, hipMalloc(&c->d_wmask, NB * kWavesPerBlock * sizeof(uint64_t)));
    LO_HIP(c, hipMalloc(&c->d_blk_cnt, NB * sizeof(int32_t)));
    LO_HIP(c, hipMalloc(&c->d_blk_sum, NB * sizeof(double)));
    LO_HIP(c, hipMalloc(&c->d_blk_m2, NB * sizeof(double)));
    LO_HIP(c, hipMalloc(&c->d_blk_part, NB * kNE * sizeof(double)));
    LO_HIP(c, hipMalloc(&c->d_js, (kMaxAlpha + 1) * sizeof(double)));
    LO_HIP(c, hipMalloc(&c->d_st, sizeof(DevState)));
    LO_HIP(c, hipHostMalloc(&c->h_st, sizeof(DevState), hipHostMallocDefault));
    std::memset(c->h_st, 0, sizeof(DevState));
    LO_HIP(c, hipHostMalloc(&c->h_nf, sizeof(int), hipHostMallocDefault));
    *c->h_nf = 0;
    LO_HIP(c, hipMemset(c->d_st, 0, sizeof(DevState)));
    // empty table (capacity 2) so a scan before any map upload finds nothing
    c->tab_cap = 2;
    c->log2cap = 1;
    LO_HIP(c, hipMalloc(&c->d_tab, c->tab_cap * sizeof(Slot)));
    LO_HIP(c, hipMemset(c->d_tab, 0xff, c->tab_cap * sizeof(Slot)));
    const int rc_t = upload_pko_tables(c, c->cfg);
    if (rc_t != LO_OK) return rc_t;
    LO_HIP(c, hipEventCreate(&c->ev0));
    LO_HIP(c, hipEventCreate(&c->ev1));
    // k_pko_t's dynamic block-prefix LDS reaches 64 KB at the 4M-point maximum
    LO_HIP(c, hipFuncSetAttribute(reinterpret_cast<const void*>(k_pko_t<4>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(kMaxBlocks * sizeof(int))));
    c->kd = g.use_surfel_correspondence == 0;
    if (c->kd) {
        int rc = kd_alloc(c);
        if (rc != LO_OK) return rc;
    }
    return LO_OK;
}

// Live contexts (a host map holding a deferred-fit ticket asks whether its context still exists).
static std::mutex g_live_mu;
static std::unordered_set<const lo_ctx*> g_live;
static uint64_t g_ticket = 0;

lo_ctx* lo_create(const lo_config* cfg, int device, int* err) {
    std::string e;
    int rc = validate_config(cfg, e);
    if (rc != LO_OK) { if (err) *err = rc; std::fprintf(stderr, "lo_create: %s\n", e.c_str()); return nullptr; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        if (err) *err = LO_ERR_HIP;
        std::fprintf(stderr, "lo_create: no HIP device %d (count %d)\n", device, ndev);
        return nullptr;
    }
    lo_ctx* c = new lo_ctx();
    c->cfg = *cfg;
    c->device = device;
    if (const char* pe = std::getenv("LO_PRESOLVE")) c->presolve = std::atoi(pe) != 0;   // A/B runs
    // rocprofv3 counter collection serialises dispatches across queues, which the pipeline's device-side waits cannot
    // survive (k_wait_final): the pipeline starts off under it unless LO_PIPE says otherwise
    if (const char* cc = std::getenv("ROCPROF_COUNTER_COLLECTION")) {
        if (*cc && std::strcmp(cc, "0") != 0 && std::strcmp(cc, "False") != 0 && std::strcmp(cc, "false") != 0) c->pipe = false;
    }
    if (const char* pp = std::getenv("LO_PIPE")) c->pipe = std::atoi(pp) != 0;
    if (const char* pm = std::getenv("LO_PIPE_MAIN")) c->pipe_main = std::max(1, std::atoi(pm));
    if (const char* pw = std::getenv("LO_PIPE_WAIT_MS")) c->pipe_bound = 100000ull * std::max(1, std::atoi(pw));
    if (const char* pf = std::getenv("LO_PIPE_FAIL_AT")) c->pipe_fail_at = static_cast<uint32_t>(std::max(0, std::atoi(pf)));
    if (const char* pg = std::getenv("LO_PKO_GROUPS")) c->pko_groups = std::max(0, std::atoi(pg));
    if (const char* ps = std::getenv("LO_PKO_SOLO")) c->pko_solo = std::atoi(ps) != 0;
    if (const char* ex = std::getenv("LO_EXACT")) c->exact = std::atoi(ex) != 0;   // A/B runs: LO_EXACT=0 = fast mode
    rc = ctx_alloc(c);
    if (rc != LO_OK) {
        std::fprintf(stderr, "lo_create: %s\n", c->err.c_str());
        lo_destroy(c);
        if (err) *err = rc;
        return nullptr;
    }
    if (err) *err = LO_OK;
    {
        std::lock_guard<std::mutex> g(g_live_mu);
        g_live.insert(c);
    }
    return c;
}

void lo_destroy(lo_ctx* c) {
    if (!c) return;
    {
        std::lock_guard<std::mutex> g(g_live_mu);
        g_live.erase(c);
    }
    (void)hipSetDevice(c->device);
    (void)sync_all(c);
    if (c->d_fin) (void)hipFree(c->d_fin);
    if (c->h_broken) (void)hipHostFree(c->h_broken);
    if (c->s_tail) (void)hipStreamDestroy(c->s_tail);
    void* bufs[] = {c->d_pts, c->d_slot, c->d_wmask, c->d_blk_cnt, c->d_blk_sum, c->d_blk_m2, c->d_blk_part, c->d_acc_part,
                    c->d_js, c->d_res, c->d_u8, c->d_st, c->d_tab, c->d_alphas, c->d_Z, c->d_tabs_i,
                    c->grid.d_pts, c->grid.d_start, c->lgrid.d_pts, c->lgrid.d_start,
                    c->grid.d_vpos, c->grid.d_nodes, c->lgrid.d_vpos, c->lgrid.d_nodes,
                    c->d_kd_nbr, c->d_kd_unres, c->d_kd_res, c->d_kd_plane, c->d_ex_terms, c->d_res_pko,
                    c->d_ex_res, c->d_ex_sorted, c->d_ex_sort_tmp, c->d_ex_tot, c->d_ex_rank,
                    c->d_mw, c->d_mwm, c->d_cand_rec, c->d_cand_cnt};
    for (void* b : bufs) if (b) (void)hipFree(b);
    if (c->grid.h_stage) (void)hipHostFree(c->grid.h_stage);
    if (c->lgrid.h_stage) (void)hipHostFree(c->lgrid.h_stage);
    if (c->d_raw) (void)hipFree(c->d_raw);
    vf_free(c->vf);
    if (c->h_st) (void)hipHostFree(c->h_st);
    if (c->h_nf) (void)hipHostFree(c->h_nf);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    for (hipEvent_t e : c->st_ev) (void)hipEventDestroy(e);
    if (c->d_span) (void)hipFree(c->d_span);
    if (c->ev_patch) (void)hipEventDestroy(c->ev_patch);
    if (c->h_patch) (void)hipHostFree(c->h_patch);
    if (c->d_patch) (void)hipFree(c->d_patch);
    if (c->ev_fit) (void)hipEventDestroy(c->ev_fit);
    if (c->h_fit_in) (void)hipHostFree(c->h_fit_in);
    if (c->d_fit_in) (void)hipFree(c->d_fit_in);
    if (c->h_fit_out) (void)hipHostFree(c->h_fit_out);
    if (c->d_fit_out) (void)hipFree(c->d_fit_out);
    if (c->stream && c->own_stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

// ---------------------------------------------------------------- map
// pack_key (lo_device.h): three 21-bit fields key + 2^20
static uint64_t pack_key_host(int32_t x, int32_t y, int32_t z) {
    return static_cast<uint64_t>(static_cast<uint32_t>(x + (1 << 20))) |
           (static_cast<uint64_t>(static_cast<uint32_t>(y + (1 << 20))) << 21) |
           (static_cast<uint64_t>(static_cast<uint32_t>(z + (1 << 20))) << 42);
}

int lo_map_set_surfels(lo_ctx* c, const int32_t* keys, const float* normals, const float* centroids, size_t m) {
    if (!c) return LO_ERR_ARG;
    if (m > 0 && (!keys || !normals || !centroids)) { c->err = "null surfel arrays"; return LO_ERR_ARG; }
    size_t cap = 2;
    uint32_t l2 = 1;
    while (cap < 4 * m) { cap <<= 1; ++l2; }            // load <= 1/4: room for in-place patches up to 1/2
    std::vector<Slot> h(cap);
    for (auto& s : h) { s.key = kEmptyKey; s.n[0] = s.n[1] = s.n[2] = 0.0f; s.c[0] = s.c[1] = s.c[2] = 0.0f; }
    const uint64_t mask = cap - 1;
    std::unordered_set<uint64_t> resident;
    resident.reserve(2 * m);
    for (size_t i = 0; i < m; ++i) {
        for (int a = 0; a < 3; ++a) {
            const int32_t v = keys[3 * i + a];
            if (v < -(1 << 20) || v >= (1 << 20)) { c->err = "surfel key outside +-2^20"; return LO_ERR_ARG; }
        }
        const uint64_t key = pack_key_host(keys[3 * i], keys[3 * i + 1], keys[3 * i + 2]);
        resident.insert(key);
        uint64_t b = (key * 0x9E3779B97F4A7C15ull) >> (64 - l2);
        while (h[b].key != kEmptyKey && h[b].key != key) b = (b + 1) & mask;
        h[b].key = key;                                    // duplicate keys: last one wins (map semantics)
        for (int a = 0; a < 3; ++a) { h[b].n[a] = normals[3 * i + a]; h[b].c[a] = centroids[3 * i + a]; }
    }
    LO_HIP(c, hipSetDevice(c->device));
    LO_HIP(c, hipStreamSynchronize(c->stream));
    if (cap > c->tab_cap) {
        LO_HIP(c, hipFree(c->d_tab));
        c->d_tab = nullptr;
        LO_HIP(c, hipMalloc(&c->d_tab, cap * sizeof(Slot)));
        c->tab_cap = cap;
    }
    LO_HIP(c, hipMemcpy(c->d_tab, h.data(), cap * sizeof(Slot), hipMemcpyHostToDevice));
    c->log2cap = l2;
    c->n_surfels = resident.size();
    c->resident.swap(resident);
    c->n_tomb = 0;
    c->map_src = 0;                                      // no longer mirrors a synced host map
    ++c->tab_gen;
    ++c->tab_edit;
    return LO_OK;
}

}  // extern "C"

namespace lo {
struct MapPatchRec {                  // one L1 voxel's change: upsert (op 1: key + payload) or erase (op 0)
    uint64_t key;
    float n[3];
    float c[3];
    uint32_t op;
    uint32_t pad;
};
void ctx_map_source(const lo_ctx* c, uint64_t* src, uint64_t* epoch, uint64_t* pos) {
    *src = c->map_src; *epoch = c->map_epoch; *pos = c->map_pos;
}
void ctx_set_map_source(lo_ctx* c, uint64_t src, uint64_t epoch, uint64_t pos) {
    c->map_src = src; c->map_epoch = epoch; c->map_pos = pos;
}

int ctx_reserve_table(lo_ctx* c, size_t min_slots, void** tab, uint32_t* log2cap, uint64_t* gen) {
    if (!c || !tab || !log2cap || !gen) return LO_ERR_ARG;
    size_t cap = 2;
    uint32_t l2 = 1;
    while (cap < min_slots) { cap <<= 1; ++l2; }
    if (c->devmap_gen != c->tab_gen || c->devmap_gen == 0 || (size_t(1) << c->log2cap) < cap) {
        LO_HIP(c, hipSetDevice(c->device));
        if (cap > c->tab_cap) {
            LO_HIP(c, hipStreamSynchronize(c->stream));
            LO_HIP(c, hipFree(c->d_tab));
            c->d_tab = nullptr;
            LO_HIP(c, hipMalloc(&c->d_tab, cap * sizeof(Slot)));
            c->tab_cap = cap;
        } else {
            cap = std::max(cap, size_t(1) << c->log2cap);   // keep the larger table
            l2 = 1;
            while ((size_t(1) << l2) < cap) ++l2;
        }
        LO_HIP(c, hipMemsetAsync(c->d_tab, 0xff, cap * sizeof(Slot), c->stream));
        c->log2cap = l2;
        c->resident.clear();
        c->n_surfels = 0;
        c->n_tomb = 0;
        c->map_src = 0;
        ++c->tab_gen;
        c->devmap_gen = c->tab_gen;
    }
    ++c->tab_edit;                                       // the device map patches the table from now on
    *tab = c->d_tab;
    *log2cap = c->log2cap;
    *gen = c->tab_gen;
    return LO_OK;
}

int ctx_filtered_device(lo_ctx* c, const float** d_pts, const int** d_n) {
    if (!c || !d_pts || !d_n) return LO_ERR_ARG;
    if (!c->last_dev_count || !c->vf.n_out) { c->err = "no device-filtered scan"; return LO_ERR_STATE; }
    *d_pts = c->d_pts;
    *d_n = c->vf.n_out;
    return LO_OK;
}

static int grow_pinned_pair(lo_ctx* c, void** h, void** d, size_t* cap, size_t bytes) {
    if (bytes <= *cap) return LO_OK;
    if (*h) LO_HIP(c, hipHostFree(*h));
    if (*d) LO_HIP(c, hipFree(*d));
    *h = *d = nullptr;
    *cap = 0;
    const size_t b = std::max<size_t>(2 * bytes, 64 * 1024);
    LO_HIP(c, hipHostMalloc(h, b, hipHostMallocDefault));
    LO_HIP(c, hipMalloc(d, b));
    *cap = b;
    return LO_OK;
}

// The pending fit launch's planarity failures leave the resident mirror (the kernel erased them from the table), once:
// before a count is reported, before another patch or fit reads the mirror, and when the map collects the results.
static int reconcile_fit(lo_ctx* c) {
    if (c->fit_ticket == 0 || c->fit_reconciled) return LO_OK;
    LO_HIP(c, hipSetDevice(c->device));
    LO_HIP(c, hipEventSynchronize(c->ev_fit));
    const FitResult* out = c->h_fit_out;
    if (c->fit_gen == c->tab_gen)                        // the table still holds what the kernel patched
        for (size_t j = 0; j < c->fit_keys.size(); ++j)
            if (out[j].planarity > c->fit_thr) c->resident.erase(c->fit_keys[j]);
    c->n_surfels = c->resident.size();
    c->fit_reconciled = true;
    return LO_OK;
}

int ctx_fit_surfels(lo_ctx* c, const int32_t* keys, const int32_t* offs, size_t n_jobs, const float* cs, size_t n_cs,
                    float thr, uint64_t* ticket) {
    if (!c || !ticket || (n_jobs > 0 && (!keys || !offs || !cs))) return LO_ERR_ARG;
    if (!c->d_tab) { c->err = "no surfel table to patch"; return LO_ERR_STATE; }
    int rc0 = reconcile_fit(c);                          // a superseded ticket's failures must not stay resident
    if (rc0 != LO_OK) return rc0;
    if (n_jobs > static_cast<size_t>(INT32_MAX) || n_cs > static_cast<size_t>(INT32_MAX / 3)) return LO_ERR_CAPACITY;
    // worst case for the table: every job not resident inserts, every resident one leaves a tombstone
    std::vector<uint64_t> pk(n_jobs);
    size_t ins = 0, ers = 0;
    for (size_t j = 0; j < n_jobs; ++j) {
        for (int a = 0; a < 3; ++a) {
            const int32_t v = keys[3 * j + a];
            if (v < -(1 << 20) || v >= (1 << 20)) { c->err = "surfel key outside +-2^20"; return LO_ERR_ARG; }
        }
        pk[j] = pack_key_host(keys[3 * j], keys[3 * j + 1], keys[3 * j + 2]);
        if (c->resident.count(pk[j])) ++ers; else ++ins;
    }
    const size_t cap = size_t(1) << c->log2cap;
    if (c->resident.size() + ins + c->n_tomb + ers > cap / 2) { c->err = "table full"; return LO_ERR_CAPACITY; }
    LO_HIP(c, hipSetDevice(c->device));
    if (!c->ev_fit) LO_HIP(c, hipEventCreateWithFlags(&c->ev_fit, hipEventDisableTiming));
    else LO_HIP(c, hipEventSynchronize(c->ev_fit));     // the previous fit has left the staging buffers
    const size_t jb = n_jobs * sizeof(FitJob), in_bytes = jb + n_cs * 3 * sizeof(float);
    int rc = grow_pinned_pair(c, &c->h_fit_in, &c->d_fit_in, &c->fit_in_cap, in_bytes);
    if (rc != LO_OK) return rc;
    void* ho = c->h_fit_out;
    void* dv = c->d_fit_out;
    rc = grow_pinned_pair(c, &ho, &dv, &c->fit_out_cap, n_jobs * sizeof(FitResult));
    c->h_fit_out = static_cast<FitResult*>(ho);
    c->d_fit_out = static_cast<FitResult*>(dv);
    if (rc != LO_OK) return rc;
    FitJob* J = static_cast<FitJob*>(c->h_fit_in);
    for (size_t j = 0; j < n_jobs; ++j) {
        const int32_t end = j + 1 < n_jobs ? offs[j + 1] : static_cast<int32_t>(n_cs);
        J[j].key = pk[j];
        J[j].off = offs[j];
        J[j].m = end - offs[j];
    }
    std::memcpy(static_cast<char*>(c->h_fit_in) + jb, cs, n_cs * 3 * sizeof(float));
    LO_HIP(c, hipMemcpyAsync(c->d_fit_in, c->h_fit_in, in_bytes, hipMemcpyHostToDevice, c->stream));
    if (n_jobs > 0)
        hipLaunchKernelGGL(k_surfel_fit, dim3(static_cast<unsigned>((n_jobs + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                           c->stream, static_cast<const FitJob*>(c->d_fit_in),
                           reinterpret_cast<const float*>(static_cast<const char*>(c->d_fit_in) + jb),
                           static_cast<int>(n_jobs), thr, c->d_tab, c->log2cap, reinterpret_cast<FitOut*>(c->d_fit_out));
    LO_HIP(c, hipGetLastError());
    LO_HIP(c, hipMemcpyAsync(c->h_fit_out, c->d_fit_out, n_jobs * sizeof(FitResult), hipMemcpyDeviceToHost, c->stream));
    LO_HIP(c, hipEventRecord(c->ev_fit, c->stream));
    {
        std::lock_guard<std::mutex> g(g_live_mu);
        c->fit_ticket = ++g_ticket;
    }
    c->fit_gen = c->tab_gen;
    ++c->tab_edit;
    c->fit_keys.swap(pk);
    c->fit_reconciled = false;
    c->fit_thr = thr;
    // until the results are collected the mirror counts every job key as resident (erases are then always sent)
    for (uint64_t k : c->fit_keys) c->resident.insert(k);
    c->n_tomb += ers;
    c->n_surfels = c->resident.size();
    *ticket = c->fit_ticket;
    return LO_OK;
}

int ctx_fit_results(lo_ctx* c, uint64_t ticket, FitResult* out, size_t n_jobs) {
    {
        std::lock_guard<std::mutex> g(g_live_mu);
        if (!c || !g_live.count(c) || c->fit_ticket != ticket || ticket == 0) return LO_ERR_STATE;
    }
    if (c->fit_keys.size() != n_jobs) return LO_ERR_STATE;
    const int rc = reconcile_fit(c);
    if (rc != LO_OK) return rc;
    std::memcpy(out, c->h_fit_out, n_jobs * sizeof(FitResult));
    c->fit_ticket = 0;
    c->fit_keys.clear();
    return LO_OK;
}
}  // namespace lo

extern "C" {

// In-place patch of the device table (the §8b lo_map_patch_surfels): upserts claim the first empty slot of their
// probe sequence (atomic CAS) or overwrite their key's payload, erases leave a tombstone that lookups probe past.
// Asynchronous on the context stream (pinned staging, no host sync).  LO_ERR_CAPACITY when live keys + tombstones
// would exceed half the table: the caller uploads the whole map instead (lo_map_set_surfels).
int lo_map_patch_surfels(lo_ctx* c, const int32_t* keys, const float* normals, const float* centroids,
                         const uint8_t* present, size_t m) {
    if (!c) return LO_ERR_ARG;
    if (m == 0) return LO_OK;
    if (!keys || !normals || !centroids || !present) { c->err = "null patch arrays"; return LO_ERR_ARG; }
    if (!c->d_tab) { c->err = "no surfel table to patch"; return LO_ERR_STATE; }
    const int rc0 = reconcile_fit(c);
    if (rc0 != LO_OK) return rc0;
    // a key given more than once: its last record wins (as lo_map_set_surfels), the earlier ones are dropped, so the
    // device patch (one thread per record) never races two records of one key.  keep[i]: record i is its key's last
    // (a sort of (key, index) instead of a per-call hash map: the keyed sync hands over a few hundred keys per keyframe)
    std::vector<std::pair<uint64_t, uint32_t>> ord(m);
    for (size_t i = 0; i < m; ++i) {
        for (int a = 0; a < 3; ++a) {
            const int32_t v = keys[3 * i + a];
            if (v < -(1 << 20) || v >= (1 << 20)) { c->err = "surfel key outside +-2^20"; return LO_ERR_ARG; }
        }
        ord[i] = {pack_key_host(keys[3 * i], keys[3 * i + 1], keys[3 * i + 2]), static_cast<uint32_t>(i)};
    }
    std::sort(ord.begin(), ord.end());
    std::vector<uint8_t> keep(m, 0), res_of(m, 0);
    size_t ins = 0, ers = 0;
    for (size_t r = 0; r < m; ++r) {
        if (r + 1 < m && ord[r + 1].first == ord[r].first) continue;   // a later record of the key follows
        const size_t i = ord[r].second;
        keep[i] = 1;
        res_of[i] = c->resident.count(ord[r].first) != 0 ? 1 : 0;
        ins += (present[i] && !res_of[i]) ? 1 : 0;
        ers += (!present[i] && res_of[i]) ? 1 : 0;
    }
    const size_t cap = size_t(1) << c->log2cap;
    if ((c->resident.size() + ins - ers) + (c->n_tomb + ers) > cap / 2) { c->err = "table full"; return LO_ERR_CAPACITY; }
    LO_HIP(c, hipSetDevice(c->device));
    const size_t bytes = m * sizeof(MapPatchRec);
    if (bytes > c->patch_cap) {
        if (c->ev_patch) LO_HIP(c, hipEventSynchronize(c->ev_patch));
        if (c->h_patch) LO_HIP(c, hipHostFree(c->h_patch));
        if (c->d_patch) LO_HIP(c, hipFree(c->d_patch));
        c->h_patch = c->d_patch = nullptr;
        const size_t cap_b = std::max<size_t>(bytes * 2, 64 * 1024);
        LO_HIP(c, hipHostMalloc(&c->h_patch, cap_b, hipHostMallocDefault));
        LO_HIP(c, hipMalloc(&c->d_patch, cap_b));
        c->patch_cap = cap_b;
    }
    if (!c->ev_patch) LO_HIP(c, hipEventCreateWithFlags(&c->ev_patch, hipEventDisableTiming));
    else LO_HIP(c, hipEventSynchronize(c->ev_patch));   // the previous patch's copy has left the staging buffer
    MapPatchRec* r = static_cast<MapPatchRec*>(c->h_patch);
    int n_rec = 0;
    for (size_t i = 0; i < m; ++i) {
        if (!keep[i]) continue;                            // superseded by a later record of the key
        const uint64_t key = pack_key_host(keys[3 * i], keys[3 * i + 1], keys[3 * i + 2]);
        const bool res = res_of[i] != 0;
        if (!present[i] && !res) continue;                 // nothing on the device to remove
        MapPatchRec& q = r[n_rec++];
        q.key = key;
        q.op = present[i] ? 1u : 0u;
        q.pad = 0;
        for (int a = 0; a < 3; ++a) { q.n[a] = normals[3 * i + a]; q.c[a] = centroids[3 * i + a]; }
        if (present[i]) c->resident.insert(key); else c->resident.erase(key);
    }
    c->n_tomb += ers;
    c->n_surfels = c->resident.size();
    if (n_rec == 0) return LO_OK;
    ++c->tab_edit;
    LO_HIP(c, hipMemcpyAsync(c->d_patch, c->h_patch, n_rec * sizeof(MapPatchRec), hipMemcpyHostToDevice, c->stream));
    LO_HIP(c, hipEventRecord(c->ev_patch, c->stream));
    hipLaunchKernelGGL(k_map_patch, dim3((n_rec + kBlock - 1) / kBlock), dim3(kBlock), 0, c->stream, c->d_tab,
                       c->log2cap, static_cast<const MapPatchRec*>(c->d_patch), n_rec);
    LO_HIP(c, hipGetLastError());
    return LO_OK;
}

// The reference-side sync: the map's whole current surfel set, diffed on the host against the set this
// context last received through this call; only the difference goes to the device (lo_map_patch_surfels: upserts of
// new / refitted surfels, erases of the ones that left).  The first call, a table changed by anything else since, or a
// full table uploads everything (lo_map_set_surfels).  *patched = records sent, -1 after a full upload.
int lo_map_sync_surfels(lo_ctx* c, const int32_t* keys, const float* normals, const float* centroids, size_t m,
                        int* patched) {
    if (!c) return LO_ERR_ARG;
    if (m > 0 && (!keys || !normals || !centroids)) { c->err = "null surfel arrays"; return LO_ERR_ARG; }
    if (c->kd) { c->err = "KDTree-mode context (lo_map_set_points)"; return LO_ERR_STATE; }
    std::unordered_map<uint64_t, size_t> in;
    in.reserve(2 * m);
    for (size_t i = 0; i < m; ++i) {
        for (int a = 0; a < 3; ++a) {
            const int32_t v = keys[3 * i + a];
            if (v < -(1 << 20) || v >= (1 << 20)) { c->err = "surfel key outside +-2^20"; return LO_ERR_ARG; }
        }
        in[pack_key_host(keys[3 * i], keys[3 * i + 1], keys[3 * i + 2])] = i;   // a repeated key: the last record
    }
    auto payload = [&](size_t i) {
        return std::array<float, 6>{normals[3 * i], normals[3 * i + 1], normals[3 * i + 2], centroids[3 * i],
                                    centroids[3 * i + 1], centroids[3 * i + 2]};
    };
    auto full = [&]() -> int {
        const int rc = lo_map_set_surfels(c, keys, normals, centroids, m);
        if (rc != LO_OK) return rc;
        c->smirror.clear();
        c->smirror.reserve(2 * in.size());
        for (const auto& kv : in) c->smirror[kv.first] = payload(kv.second);
        c->mirror_edit = c->tab_edit;
        if (patched) *patched = -1;
        return LO_OK;
    };
    if (c->mirror_edit != c->tab_edit) return full();
    std::vector<int32_t> pk;
    std::vector<float> pn, pc;
    std::vector<uint8_t> pres;
    for (const auto& kv : in) {
        const std::array<float, 6> p = payload(kv.second);
        auto it = c->smirror.find(kv.first);
        if (it != c->smirror.end() && std::memcmp(it->second.data(), p.data(), sizeof(p)) == 0) continue;   // unchanged
        const size_t i = kv.second;
        pk.insert(pk.end(), {keys[3 * i], keys[3 * i + 1], keys[3 * i + 2]});
        pn.insert(pn.end(), {p[0], p[1], p[2]});
        pc.insert(pc.end(), {p[3], p[4], p[5]});
        pres.push_back(1);
    }
    for (const auto& kv : c->smirror) {
        if (in.count(kv.first)) continue;                 // still a surfel
        const uint64_t k = kv.first;
        pk.insert(pk.end(), {static_cast<int32_t>(k & 0x1FFFFF) - (1 << 20), static_cast<int32_t>((k >> 21) & 0x1FFFFF) - (1 << 20),
                             static_cast<int32_t>((k >> 42) & 0x1FFFFF) - (1 << 20)});
        pn.insert(pn.end(), {0.0f, 0.0f, 0.0f});
        pc.insert(pc.end(), {0.0f, 0.0f, 0.0f});
        pres.push_back(0);
    }
    const size_t np = pres.size();
    if (np == 0) { if (patched) *patched = 0; return LO_OK; }
    const int rc = lo_map_patch_surfels(c, pk.data(), pn.data(), pc.data(), pres.data(), np);
    if (rc == LO_ERR_CAPACITY) return full();            // tombstones / growth: rebuild the table
    if (rc != LO_OK) return rc;
    for (size_t r = 0; r < np; ++r) {
        const uint64_t k = pack_key_host(pk[3 * r], pk[3 * r + 1], pk[3 * r + 2]);
        if (pres[r]) c->smirror[k] = {pn[3 * r], pn[3 * r + 1], pn[3 * r + 2], pc[3 * r], pc[3 * r + 1], pc[3 * r + 2]};
        else c->smirror.erase(k);
    }
    c->mirror_edit = c->tab_edit;
    if (patched) *patched = static_cast<int>(np);
    return LO_OK;
}

// IterativeClosestPointOptimizer::update_config (IterativeClosestPointOptimizer.h:220) replaces the parameters and
// nothing else: the device map, the scan buffers and the stream stay.  The layout fields (voxel geometry, max_points,
// correspondence mode) size or key those and cannot change here.  New PKO parameters rebuild the PKO tables.
int lo_update_config(lo_ctx* c, const lo_config* cfg) {
    if (!c) return LO_ERR_ARG;
    std::string e;
    int rc = validate_config(cfg, e);
    if (rc != LO_OK) { c->err = e; return rc; }
    const lo_config& o = c->cfg;
    if (cfg->voxel_size != o.voxel_size || cfg->hierarchy_factor != o.hierarchy_factor || cfg->max_points != o.max_points ||
        cfg->use_surfel_correspondence != o.use_surfel_correspondence) {
        c->err = "update_config: voxel_size / hierarchy_factor / max_points / use_surfel_correspondence are fixed at lo_create";
        return LO_ERR_STATE;
    }
    LO_HIP(c, hipSetDevice(c->device));
    LO_HIP(c, sync_all(c));
    const bool pko_changed = cfg->gmm_sample_size != o.gmm_sample_size || cfg->gmm_components != o.gmm_components ||
                             cfg->min_scale_factor != o.min_scale_factor || cfg->max_scale_factor != o.max_scale_factor ||
                             cfg->num_alpha_segments != o.num_alpha_segments ||
                             cfg->truncated_threshold != o.truncated_threshold || cfg->pko_kernel != o.pko_kernel;
    const bool na_changed = cfg->num_alpha_segments != o.num_alpha_segments;
    if (pko_changed) {                                   // the new tables first: a failure leaves the context unchanged
        rc = upload_pko_tables(c, *cfg);
        if (rc != LO_OK) return rc;
    }
    c->cfg = *cfg;
    ++c->cfg_gen;                                        // batches re-upload this context's parameters
    if (na_changed || (cfg->use_adaptive_m_estimator && !c->d_acc_part)) {
        // the candidate buffers are sized by the alpha grid: re-made on the next optimize
        if (c->d_acc_part) LO_HIP(c, hipFree(c->d_acc_part));
        if (c->d_cand_rec) LO_HIP(c, hipFree(c->d_cand_rec));
        if (c->d_cand_cnt) LO_HIP(c, hipFree(c->d_cand_cnt));
        c->d_acc_part = nullptr;
        c->d_cand_rec = nullptr;
        c->d_cand_cnt = nullptr;
    }
    return LO_OK;
}

size_t lo_map_surfel_count(const lo_ctx* c) {
    if (!c) return 0;
    lo_ctx* w = const_cast<lo_ctx*>(c);
    if (reconcile_fit(w) != LO_OK) return 0;             // pending device fits: count their planarity failures out
    return w->n_surfels;
}

// VoxelMap::RebuildKdTree (VoxelMap.cpp:420-438) equivalent: a dense uniform grid (cell = 2 x voxel, doubled
// until it fits kKdMaxCells) over the L0 centroids in GetPointCloud order; points sorted by cell (x fastest),
// index order inside a cell; kd_start[cell] = first point, kd_start[ncell] = m.
static constexpr size_t kKdMaxCells = size_t(1) << 26;

// with_order: also the reference kd-tree's visit order (the tie-break of equal distances); without it the kNN
// kernels flag a deciding tie in DevState::kd_tie instead of ranking it (the loop-closure ICP then rebuilds with it).
// min_per_cell > 0 (the loop-closure ICP's matched keyframe cloud): the cell edge doubles (up to 3 times) while the
// occupied cells hold fewer than min_per_cell points on average -- a voxel-filtered, strided keyframe cloud is sparse
// at 2 x voxel_size, so most queries would need the outer shells or the brute-force fallback.  The kNN result does
// not depend on the edge (every answer is certified against the scanned cube); only the work per query does.
static int grid_build(lo_ctx* c, PointGrid& G, const float* xyz, size_t m, bool with_order = true, int min_per_cell = 0) {
    if (m > 0 && !xyz) { c->err = "null points"; return LO_ERR_ARG; }
    if (m > static_cast<size_t>(INT32_MAX / 2)) { c->err = "too many map points"; return LO_ERR_CAPACITY; }
    for (size_t i = 0; i < 3 * m; ++i)
        if (!std::isfinite(xyz[i])) { c->err = "non-finite map point"; return LO_ERR_ARG; }
    // the reference kd-tree's visit order over the same cloud (equal-distance neighbours are ranked by it): built
    // on a second host thread while this one builds the grid (nanoflann's partition passes are branch-bound,
    // ~0.3 ms for a 3.6k-point keyframe cloud, as the reference's own buildIndex per loop-closure call)
    std::vector<KdNode> nodes;
    std::vector<uint32_t> vpos;
    std::thread order_thread([&] { if (with_order) KdOrderBuilder(xyz, m).build(nodes, vpos); });
    struct Joiner { std::thread& t; ~Joiner() { if (t.joinable()) t.join(); } } joiner{order_thread};
    float h = 2.0f * c->cfg.voxel_size;
    int org[3] = {0, 0, 0}, dim[3] = {1, 1, 1};
    auto cell = [&](float v) { return static_cast<int64_t>(std::floor(v / h)); };
    std::vector<uint32_t> start, lin(m);
    for (int grow = 0;; ++grow) {
    for (;;) {
        int64_t lo[3] = {INT64_MAX, INT64_MAX, INT64_MAX}, hi[3] = {INT64_MIN, INT64_MIN, INT64_MIN};
        for (size_t i = 0; i < m; ++i)
            for (int a = 0; a < 3; ++a) { const int64_t k = cell(xyz[3 * i + a]); lo[a] = std::min(lo[a], k); hi[a] = std::max(hi[a], k); }
        if (m == 0) { for (int a = 0; a < 3; ++a) { lo[a] = 0; hi[a] = 0; } }
        size_t ncell = 1;
        bool ok = true;
        for (int a = 0; a < 3; ++a) {
            const int64_t d = hi[a] - lo[a] + 1;
            if (d > static_cast<int64_t>(kKdMaxCells) || lo[a] < INT32_MIN / 2 || hi[a] > INT32_MAX / 2) { ok = false; break; }
            ncell *= static_cast<size_t>(d);
            if (ncell > kKdMaxCells) { ok = false; break; }
        }
        if (ok) { for (int a = 0; a < 3; ++a) { org[a] = static_cast<int>(lo[a]); dim[a] = static_cast<int>(hi[a] - lo[a] + 1); } break; }
        h *= 2.0f;
    }
    const size_t ncell = static_cast<size_t>(dim[0]) * dim[1] * dim[2];
    start.assign(ncell + 1, 0);
    size_t occupied = 0;
    for (size_t i = 0; i < m; ++i) {
        const int64_t x = cell(xyz[3 * i]) - org[0], y = cell(xyz[3 * i + 1]) - org[1], z = cell(xyz[3 * i + 2]) - org[2];
        lin[i] = static_cast<uint32_t>((static_cast<size_t>(z) * dim[1] + y) * dim[0] + x);
        occupied += start[lin[i] + 1]++ == 0;
    }
    if (min_per_cell > 0 && grow < 3 && m >= 64 && occupied * static_cast<size_t>(min_per_cell) > m) { h *= 2.0f; continue; }
    break;
    }
    const size_t ncell = static_cast<size_t>(dim[0]) * dim[1] * dim[2];
    for (size_t k = 0; k < ncell; ++k) start[k + 1] += start[k];
    std::vector<float4> pts(std::max<size_t>(m, 1));
    std::vector<uint32_t> fill(start.begin(), start.end() - 1);
    for (size_t i = 0; i < m; ++i) {                     // stable: index order inside a cell
        float4 v;
        v.x = xyz[3 * i]; v.y = xyz[3 * i + 1]; v.z = xyz[3 * i + 2];
        int32_t id = static_cast<int32_t>(i);
        std::memcpy(&v.w, &id, sizeof(float));
        pts[fill[lin[i]]++] = v;
    }
    LO_HIP(c, hipSetDevice(c->device));
    LO_HIP(c, hipStreamSynchronize(c->stream));
    if (pts.size() > G.pts_cap) {
        if (G.d_pts) LO_HIP(c, hipFree(G.d_pts));
        G.d_pts = nullptr;
        LO_HIP(c, hipMalloc(&G.d_pts, pts.size() * sizeof(float4)));
        G.pts_cap = pts.size();
    }
    if (start.size() > G.start_cap) {
        if (G.d_start) LO_HIP(c, hipFree(G.d_start));
        G.d_start = nullptr;
        LO_HIP(c, hipMalloc(&G.d_start, start.size() * sizeof(uint32_t)));
        G.start_cap = start.size();
    }
    order_thread.join();
    if (nodes.empty()) nodes.push_back(KdNode{-1, -1, 0, 0, 0.0f, 0.0f});
    if (vpos.empty()) vpos.push_back(0);
    if (vpos.size() > G.vpos_cap) {
        if (G.d_vpos) LO_HIP(c, hipFree(G.d_vpos));
        G.d_vpos = nullptr;
        LO_HIP(c, hipMalloc(&G.d_vpos, vpos.size() * sizeof(uint32_t)));
        G.vpos_cap = vpos.size();
    }
    if (nodes.size() > G.nodes_cap) {
        if (G.d_nodes) LO_HIP(c, hipFree(G.d_nodes));
        G.d_nodes = nullptr;
        LO_HIP(c, hipMalloc(&G.d_nodes, nodes.size() * sizeof(KdNode)));
        G.nodes_cap = nodes.size();
    }
    // one pinned staging buffer, four async copies on the context stream (the kernels that read the grid follow
    // in stream order; the next grid_build's stream sync retires the copies before the buffer is refilled)
    const size_t b_pts = pts.size() * sizeof(float4), b_start = start.size() * sizeof(uint32_t);
    const size_t b_vpos = vpos.size() * sizeof(uint32_t), b_nodes = nodes.size() * sizeof(KdNode);
    const size_t total = b_pts + b_start + b_vpos + b_nodes;
    if (total > G.stage_cap) {
        if (G.h_stage) LO_HIP(c, hipHostFree(G.h_stage));
        G.h_stage = nullptr;
        G.stage_cap = 0;
        LO_HIP(c, hipHostMalloc(&G.h_stage, 2 * total, hipHostMallocDefault));
        G.stage_cap = 2 * total;
    }
    char* hs = static_cast<char*>(G.h_stage);
    std::memcpy(hs, pts.data(), b_pts);
    std::memcpy(hs + b_pts, start.data(), b_start);
    std::memcpy(hs + b_pts + b_start, vpos.data(), b_vpos);
    std::memcpy(hs + b_pts + b_start + b_vpos, nodes.data(), b_nodes);
    LO_HIP(c, hipMemcpyAsync(G.d_pts, hs, b_pts, hipMemcpyHostToDevice, c->stream));
    LO_HIP(c, hipMemcpyAsync(G.d_start, hs + b_pts, b_start, hipMemcpyHostToDevice, c->stream));
    LO_HIP(c, hipMemcpyAsync(G.d_vpos, hs + b_pts + b_start, b_vpos, hipMemcpyHostToDevice, c->stream));
    LO_HIP(c, hipMemcpyAsync(G.d_nodes, hs + b_pts + b_start + b_vpos, b_nodes, hipMemcpyHostToDevice, c->stream));
    G.m = static_cast<int>(m);
    G.has_order = with_order;
    G.all = false;
    G.h = h;
    for (int a = 0; a < 3; ++a) { G.org[a] = org[a]; G.dim[a] = dim[a]; }
    return LO_OK;
}

// A small point set (<= kKnnAllMax) for the all-pairs kernels (k_knn_all, k_inlier_all): the points in index order as
// float4 (x, y, z, index), no cells and no visit order; with q (nq points) also the query cloud into c->d_pts, both
// through the grid's pinned staging buffer (two async copies, no pageable-memory copy).
static int all_pairs_upload(lo_ctx* c, PointGrid& G, const float* xyz, size_t m, const float* q = nullptr, size_t nq = 0) {
    if (m > static_cast<size_t>(kKnnAllMax)) { c->err = "all_pairs_upload: too many points"; return LO_ERR_CAPACITY; }
    if (m > 0 && !xyz) { c->err = "null points"; return LO_ERR_ARG; }
    for (size_t i = 0; i < 3 * m; ++i)
        if (!std::isfinite(xyz[i])) { c->err = "non-finite map point"; return LO_ERR_ARG; }
    LO_HIP(c, hipSetDevice(c->device));
    LO_HIP(c, hipStreamSynchronize(c->stream));          // the staging buffer's previous copy has retired
    const size_t mm = std::max<size_t>(m, 1), bytes = mm * sizeof(float4) + nq * 3 * sizeof(float);
    if (mm > G.pts_cap) {
        if (G.d_pts) LO_HIP(c, hipFree(G.d_pts));
        G.d_pts = nullptr;
        LO_HIP(c, hipMalloc(&G.d_pts, bytes));
        G.pts_cap = mm;
    }
    if (bytes > G.stage_cap) {
        if (G.h_stage) LO_HIP(c, hipHostFree(G.h_stage));
        G.h_stage = nullptr;
        G.stage_cap = 0;
        LO_HIP(c, hipHostMalloc(&G.h_stage, 2 * bytes, hipHostMallocDefault));
        G.stage_cap = 2 * bytes;
    }
    float4* hs = static_cast<float4*>(G.h_stage);
    for (size_t i = 0; i < m; ++i) {
        int32_t id = static_cast<int32_t>(i);
        float w;
        std::memcpy(&w, &id, sizeof(float));
        hs[i] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], w);
    }
    if (m > 0) LO_HIP(c, hipMemcpyAsync(G.d_pts, hs, m * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    if (nq > 0) {
        float* hq = reinterpret_cast<float*>(hs + mm);
        std::memcpy(hq, q, nq * 3 * sizeof(float));
        LO_HIP(c, hipMemcpyAsync(c->d_pts, hq, nq * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    }
    G.m = static_cast<int>(m);
    G.has_order = false;
    G.all = true;
    return LO_OK;
}

}  // extern "C"

namespace lo {
// ---- the same grid built on the device (ctx_grid_from_device: the device map's L0 centroids) ----
// Every kernel here clamps the device count to the array's capacity: a corrupt or overflowing count is reported by the
// host (out[6] carries the raw count) without a read past the array.
__global__ __launch_bounds__(1024) void k_grid_bounds(const float* __restrict__ xyz, const int* __restrict__ d_count,
                                                     int cap, float* __restrict__ out) {
    __shared__ float s[6][16];
    const int m_raw = *d_count, m = min(max(m_raw, 0), cap), tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = tid; i < m; i += 1024)
        for (int a = 0; a < 3; ++a) { const float v = xyz[3 * i + a]; lo[a] = fminf(lo[a], v); hi[a] = fmaxf(hi[a], v); }
    for (int o = 32; o > 0; o >>= 1)
        for (int a = 0; a < 3; ++a) { lo[a] = fminf(lo[a], __shfl_xor(lo[a], o, 64)); hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], o, 64)); }
    if (lane == 0) for (int a = 0; a < 3; ++a) { s[a][wid] = lo[a]; s[3 + a][wid] = hi[a]; }
    __syncthreads();
    if (tid < 6) {
        float r = s[tid][0];
        for (int w = 1; w < 16; ++w) r = tid < 3 ? fminf(r, s[tid][w]) : fmaxf(r, s[tid][w]);
        out[tid] = r;
    }
    if (tid == 0) out[6] = __int_as_float(m_raw);
}
struct GridGeom {
    float h;
    int org[3], dim[3];
};
// grid_build's cell of a coordinate: floor(v / h) in fp32, as an int64 (the same operations)
__device__ __forceinline__ long long grid_cell(float v, float h) { return static_cast<long long>(floorf(v / h)); }
__global__ void k_grid_keys(const float* __restrict__ xyz, const int* __restrict__ d_count, int cap, GridGeom g,
                            uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, uint32_t* __restrict__ counts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= min(*d_count, cap)) return;
    const long long x = grid_cell(xyz[3 * i], g.h) - g.org[0], y = grid_cell(xyz[3 * i + 1], g.h) - g.org[1],
                    z = grid_cell(xyz[3 * i + 2], g.h) - g.org[2];
    const uint32_t lin = static_cast<uint32_t>((static_cast<unsigned long long>(z) * g.dim[1] + y) * g.dim[0] + x);
    keys[i] = lin;
    vals[i] = static_cast<uint32_t>(i);
    atomicAdd(&counts[lin], 1u);
}
__global__ void k_grid_scatter(const float* __restrict__ xyz, const int* __restrict__ d_count, int cap,
                               const uint32_t* __restrict__ svals, float4* __restrict__ pts) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= min(*d_count, cap)) return;
    const uint32_t i = svals[p];
    pts[p] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], __int_as_float(static_cast<int>(i)));
}

int ctx_grid_from_device(lo_ctx* c, const float* d_xyz, const int* d_count, size_t cap) {
    if (!c || !d_xyz || !d_count) return LO_ERR_ARG;
    if (!c->kd) { c->err = "ctx_grid_from_device: a KDTree-mode context"; return LO_ERR_STATE; }
    LO_HIP(c, hipSetDevice(c->device));
    PointGrid& G = c->grid;
    DevGridScratch& S = c->gscr;
    if (!S.d_bounds) LO_HIP(c, hipMalloc(&S.d_bounds, 8 * sizeof(float)));
    if (!S.h_bounds) LO_HIP(c, hipHostMalloc(&S.h_bounds, 8 * sizeof(float), hipHostMallocDefault));
    const int capi = static_cast<int>(std::min(cap, static_cast<size_t>(INT32_MAX)));
    hipLaunchKernelGGL(k_grid_bounds, dim3(1), dim3(1024), 0, c->stream, d_xyz, d_count, capi, S.d_bounds);
    LO_HIP(c, hipMemcpyAsync(S.h_bounds, S.d_bounds, 8 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    LO_HIP(c, hipStreamSynchronize(c->stream));
    int mi = 0;
    std::memcpy(&mi, &S.h_bounds[6], sizeof(int));
    const size_t m = static_cast<size_t>(std::max(mi, 0));
    if (m > cap) { c->err = "ctx_grid_from_device: count beyond the array"; return LO_ERR_CAPACITY; }
    // grid_build's geometry loop, from the bounds (floor(v / h) is monotone in v, so the cells' extremes are the
    // extremes' cells)
    float h = 2.0f * c->cfg.voxel_size;
    int org[3] = {0, 0, 0}, dim[3] = {1, 1, 1};
    auto cell = [&](float v) { return static_cast<int64_t>(std::floor(v / h)); };
    for (;;) {
        int64_t lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            lo[a] = m ? cell(S.h_bounds[a]) : 0;
            hi[a] = m ? cell(S.h_bounds[3 + a]) : 0;
        }
        size_t ncell = 1;
        bool ok = true;
        for (int a = 0; a < 3; ++a) {
            const int64_t d = hi[a] - lo[a] + 1;
            if (d > static_cast<int64_t>(kKdMaxCells) || lo[a] < INT32_MIN / 2 || hi[a] > INT32_MAX / 2) { ok = false; break; }
            ncell *= static_cast<size_t>(d);
            if (ncell > kKdMaxCells) { ok = false; break; }
        }
        if (ok) { for (int a = 0; a < 3; ++a) { org[a] = static_cast<int>(lo[a]); dim[a] = static_cast<int>(hi[a] - lo[a] + 1); } break; }
        h *= 2.0f;
    }
    const size_t ncell = static_cast<size_t>(dim[0]) * dim[1] * dim[2];
    auto grow = [&](auto*& p, size_t& capv, size_t need) -> int {
        if (need <= capv) return LO_OK;
        if (p) LO_HIP(c, hipFree(p));
        p = nullptr;
        LO_HIP(c, hipMalloc(&p, need * sizeof(*p)));
        capv = need;
        return LO_OK;
    };
    const size_t mm = std::max<size_t>(m, 1);
    int rc;
    if ((rc = grow(G.d_pts, G.pts_cap, mm)) != LO_OK) return rc;
    if ((rc = grow(G.d_start, G.start_cap, ncell + 1)) != LO_OK) return rc;
    if ((rc = grow(S.d_keys, S.keys_cap, 4 * mm)) != LO_OK) return rc;       // keys, vals, sorted keys, sorted vals
    if ((rc = grow(S.d_counts, S.counts_cap, ncell + 1)) != LO_OK) return rc;
    uint32_t *keys = S.d_keys, *vals = keys + mm, *skeys = vals + mm, *svals = skeys + mm;
    int bits = 1;
    while (bits < 32 && (size_t(1) << bits) < ncell) ++bits;
    size_t tmp_sort = 0, tmp_scan = 0;
    LO_HIP(c, hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_sort, keys, skeys, vals, svals, static_cast<int>(mm), 0, bits,
                                                 c->stream));
    LO_HIP(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_scan, S.d_counts, G.d_start, static_cast<int>(ncell + 1),
                                               c->stream));
    if ((rc = grow(S.d_tmp, S.tmp_cap, std::max(tmp_sort, tmp_scan))) != LO_OK) return rc;
    LO_HIP(c, hipMemsetAsync(S.d_counts, 0, (ncell + 1) * sizeof(uint32_t), c->stream));
    GridGeom g{h, {org[0], org[1], org[2]}, {dim[0], dim[1], dim[2]}};
    if (m > 0) {
        const dim3 grid((m + 255) / 256), blk(256);
        hipLaunchKernelGGL(k_grid_keys, grid, blk, 0, c->stream, d_xyz, d_count, capi, g, keys, vals, S.d_counts);
        size_t t = S.tmp_cap;
        LO_HIP(c, hipcub::DeviceRadixSort::SortPairs(S.d_tmp, t, keys, skeys, vals, svals, static_cast<int>(m), 0, bits,
                                                     c->stream));
        hipLaunchKernelGGL(k_grid_scatter, grid, blk, 0, c->stream, d_xyz, d_count, capi, svals, G.d_pts);
    }
    size_t t2 = S.tmp_cap;                               // start[cell] = points in the cells before it; start[ncell] = m
    LO_HIP(c, hipcub::DeviceScan::ExclusiveSum(S.d_tmp, t2, S.d_counts, G.d_start, static_cast<int>(ncell + 1), c->stream));
    LO_HIP(c, hipGetLastError());
    G.m = static_cast<int>(m);
    G.has_order = false;
    G.all = false;
    G.h = h;
    for (int a = 0; a < 3; ++a) { G.org[a] = org[a]; G.dim[a] = dim[a]; }
    c->grid_dev = true;
    return LO_OK;
}

}  // namespace lo

extern "C" {

int lo_map_set_points(lo_ctx* c, const float* xyz, size_t m) {
    if (!c) return LO_ERR_ARG;
    if (!c->kd) { c->err = "lo_map_set_points needs use_surfel_correspondence = 0"; return LO_ERR_STATE; }
    c->grid_dev = false;
    return grid_build(c, c->grid, xyz, m);
}

// The kd visit order for a device-built grid (ctx_grid_from_device): its points back in index order (each grid
// point carries its index), then the host build with the order -- the same grid plus the order.
static int grid_add_order(lo_ctx* c) {
    PointGrid& G = c->grid;
    const size_t m = static_cast<size_t>(G.m);
    std::vector<float4> p(std::max<size_t>(m, 1));
    LO_HIP(c, hipStreamSynchronize(c->stream));
    if (m > 0) LO_HIP(c, hipMemcpy(p.data(), G.d_pts, m * sizeof(float4), hipMemcpyDeviceToHost));
    std::vector<float> xyz(3 * std::max<size_t>(m, 1));
    for (size_t k = 0; k < m; ++k) {
        int i;
        std::memcpy(&i, &p[k].w, sizeof(int));
        if (i < 0 || static_cast<size_t>(i) >= m) { c->err = "device grid: bad point index"; return LO_ERR_STATE; }
        xyz[3 * i] = p[k].x; xyz[3 * i + 1] = p[k].y; xyz[3 * i + 2] = p[k].z;
    }
    const int rc = grid_build(c, G, xyz.data(), m, true);
    if (rc == LO_OK) c->grid_dev = true;                 // still the device map's grid (the next keyframe rebuilds it)
    return rc;
}

int lo_kd_reruns(const lo_ctx* c) { return c ? c->kd_reruns : -1; }

size_t lo_map_point_count(const lo_ctx* c) { return c ? static_cast<size_t>(c->grid.m) : 0; }

// ---------------------------------------------------------------- optimize
// Correspondence stage of one GN iteration: surfel lookup, or (KDTree variant) grid kNN + brute-force
// fallback + plane fit.  P0 carries init = 1 on a scan's first iteration.
static constexpr int kBruteBlocks = 64;      // k_knn_brute workgroups (grid-strided over the unresolved list)
static constexpr int kBruteWaveBlocks = 256; // k_knn_brute_w: 4 queries in flight per workgroup
static constexpr int kBruteWaveMaxM = 16384; // k_knn_brute_w up to this many grid points (<= 256 per lane)

// The unresolved queries: a wave per query (k_knn_brute_w) over a small grid without the kd visit order, else a
// 1024-thread workgroup per query (k_knn_brute, which also ranks deciding ties in the visit order when it is built).
static void launch_brute(lo_ctx* c, const KParams& P) {
    if (!P.kd_nodes && P.kd_m <= kBruteWaveMaxM) hipLaunchKernelGGL(k_knn_brute_w, dim3(kBruteWaveBlocks), dim3(kBlock), 0, c->stream, P);
    else hipLaunchKernelGGL(k_knn_brute, dim3(kBruteBlocks), dim3(1024), 0, c->stream, P);
}

static dim3 knn_grid(const KParams& P) { return dim3((static_cast<size_t>(P.n) * kKnnGroup + kBlock - 1) / kBlock); }
static size_t all_lds(const KParams& P) { return static_cast<size_t>((std::max(P.kd_m, 1) + 511) / 512 * 512) * sizeof(float4); }   // all_padded
static dim3 all_grid(const KParams& P) { return dim3((std::max(P.n, 1) + kAllThreads / 64 - 1) / (kAllThreads / 64)); }

static void launch_correspond(lo_ctx* c, const KParams& P, int with_stats, bool kd) {
    const dim3 grid(P.nb), blk(kBlock);
    if (!kd) {
        hipLaunchKernelGGL(k_correspond, grid, blk, 0, c->stream, P, with_stats);
        return;
    }
    KParams Pn = P;
    Pn.init = 0;
    if (P.kd_all) {                                      // a small set searched whole from LDS: no fallback pass
        hipLaunchKernelGGL(k_knn_all, all_grid(P), dim3(kAllThreads), all_lds(P), c->stream, P);
        hipLaunchKernelGGL(k_plane, grid, blk, 0, c->stream, Pn, with_stats);
        return;
    }
    hipLaunchKernelGGL(k_knn, knn_grid(P), blk, 0, c->stream, P);
    launch_brute(c, Pn);
    hipLaunchKernelGGL(k_plane, grid, blk, 0, c->stream, Pn, with_stats);
}

// After a KDTree-variant PKO launch (small scans): the iteration's solve -- the selected candidate's record
// (k_pick_knn) or its partial sums solved in every block (k_solve_knn) -- fused with the kNN search of it + 1, then
// the unresolved queries and the plane stage.
static void launch_pick_knn(lo_ctx* c, const KParams& P, int it) {
    const dim3 knn = knn_grid(P), blk(kBlock);
    if (P.kd_all) {
        if (P.cand_rec) {
            hipLaunchKernelGGL(k_pick_knn_all, all_grid(P), dim3(kAllThreads), all_lds(P), c->stream, P, it);
        } else {
            hipLaunchKernelGGL(k_solve_pick, dim3(1), blk, 0, c->stream, P, it);
            hipLaunchKernelGGL(k_knn_all, all_grid(P), dim3(kAllThreads), all_lds(P), c->stream, P);
        }
        hipLaunchKernelGGL(k_plane, dim3(P.nb), blk, 0, c->stream, P, 0);
        return;
    }
    if (P.cand_rec) hipLaunchKernelGGL(k_pick_knn, knn, blk, 0, c->stream, P, it);
    else hipLaunchKernelGGL(k_solve_knn, knn, blk, 0, c->stream, P, it);
    launch_brute(c, P);
    hipLaunchKernelGGL(k_plane, dim3(P.nb), blk, 0, c->stream, P, 0);
}

static constexpr int kStageEvents = 1024;
static constexpr int kExactMaxPoints = 16384;         // reference-exact mode: one-workgroup sort in LDS up to here
static_assert(kExactMaxPoints >= 2 * kExactMergeMax, "d_ex_rank holds the presorted runs and the merged keys");

// A scan's first correspondence launch, bracketed by HIP events on the context stream when stage timing is on
// (the kernel's in-step duration, as opposed to lo_bench_kernel's back-to-back launches).
static void launch_correspond_first(lo_ctx* c, const KParams& P0, bool kd, int with_stats = 1) {
    const bool timed = c->stage_timing && c->st_n < kStageEvents;
    if (timed) (void)hipEventRecord(c->st_ev[2 * c->st_n], c->stream);
    if (timed && !kd && c->d_span) {                     // and its own execution span (k_correspond, P.span)
        KParams Pt = P0;
        Pt.span = c->d_span + static_cast<size_t>(kSpanWords) * c->st_n;
        launch_correspond(c, Pt, with_stats, kd);
    } else {
        launch_correspond(c, P0, with_stats, kd);
    }
    if (timed) (void)hipEventRecord(c->st_ev[2 * c->st_n++ + 1], c->stream);
}

// Reference-exact mode (lo_exact.hip): device buffers on first use, then per GN iteration the correspondence stage,
// (iteration 0) the sorted-order scale, the PKO, the per-point terms and the sequential sums + fp32 solve.  Scans of
// at most kExactMaxPoints sort in one workgroup (*n2 = n: registers + LDS, lo_seqsum.h); larger scans (*n2 = 0)
// write their residuals out, sort them with hipCUB's radix sort and sum them across the chip (launch_mwm_scale).
static int exact_prepare(lo_ctx* c, KParams& P, size_t n, int* n2) {
    // the term buffer: row-major [point][43] up to kExactMaxPoints (k_exact_terms + k_exact_solve), term-major rows of
    // round_up(n, 64) beyond (the 14 factor rows, or the 43 term columns in the LO_EXACT_FACTORED=0 A/B build)
    const size_t ex_need = std::max(static_cast<size_t>(kExactMaxPoints) * kExactTerms,
                                    (kExactFactored ? kExactFactors : kExactTerms) * ((n + 63) & ~static_cast<size_t>(63)));
    if (!c->d_ex_terms || c->ex_cap < ex_need) {
        if (c->d_ex_terms) LO_HIP(c, hipFree(c->d_ex_terms));
        c->d_ex_terms = nullptr;
        c->ex_cap = ex_need;
        LO_HIP(c, hipMalloc(&c->d_ex_terms, c->ex_cap * sizeof(float)));
    }
    if (!c->d_ex_rank) LO_HIP(c, hipMalloc(&c->d_ex_rank, kExactMaxPoints * sizeof(double)));
    if (!c->ex_attr) {
        LO_HIP(c, exact_scale_rank_prepare());
        LO_HIP(c, exact_scale_m_prepare());
        LO_HIP(c, exact_scale_c_prepare());
        c->ex_attr = true;
    }
    P.ex_terms = c->d_ex_terms;
    P.scale_given = 1;
    // up to kExactMergeMax points the iteration-0 correspondence launch presorts its blocks (P0.presort, set by the
    // caller from ex_merge) and one workgroup merges and sums them
    // (r06: up to kExactMaxPoints; a device-counted scan -- the voxel filter's output -- picks its sort width from the
    // count on the device, k_exact_scale_cd, instead of sizing the sort by the bound ceil(n_raw / stride))
    c->ex_merge = n <= static_cast<size_t>(kExactMaxPoints);
    c->ex_merge_presort = n <= static_cast<size_t>(kExactMergeMax) && std::getenv("LO_EXACT_PRESORT") != nullptr;   // A/B
    if (std::getenv("LO_EXACT_RANKSORT")) c->ex_merge = c->ex_merge_presort = false;   // A/B: the chip-wide rank sort
    if (n > static_cast<size_t>(kExactMaxPoints)) {
        if (!c->d_ex_tot) LO_HIP(c, hipMalloc(&c->d_ex_tot, 64 * sizeof(float)));
        if (c->mw_n_cap < n) {                               // the column sums' head records
            if (c->d_mw) LO_HIP(c, hipFree(c->d_mw));
            c->d_mw = nullptr;
            c->mw_n_cap = n;
            LO_HIP(c, hipMalloc(&c->d_mw, mw_bytes(43, static_cast<int>(n))));
            c->mw = mw_layout(c->d_mw, 43, static_cast<int>(n));
            LO_HIP(c, mw_clear(c->mw, 43, c->stream));
            LO_HIP(c, hipStreamSynchronize(c->stream));
            if (c->d_mwm) LO_HIP(c, hipFree(c->d_mwm));
            c->d_mwm = nullptr;
            LO_HIP(c, hipMalloc(&c->d_mwm, mwm_bytes(static_cast<int>(n))));
            c->mwm = mwm_layout(c->d_mwm, static_cast<int>(n));
        }
        P.ex_ld = static_cast<int>((n + 63) & ~static_cast<size_t>(63));   // term-major rows, 256-B aligned
        P.ex_tot = c->d_ex_tot;
        if (c->ex_res_cap < n) {
            if (c->d_ex_res) LO_HIP(c, hipFree(c->d_ex_res));
            if (c->d_ex_sorted) LO_HIP(c, hipFree(c->d_ex_sorted));
            if (c->d_ex_sort_tmp) LO_HIP(c, hipFree(c->d_ex_sort_tmp));
            c->d_ex_res = c->d_ex_sorted = nullptr;
            c->d_ex_sort_tmp = nullptr;
            c->ex_res_cap = n;
            LO_HIP(c, hipMalloc(&c->d_ex_res, n * sizeof(double)));
            LO_HIP(c, hipMalloc(&c->d_ex_sorted, n * sizeof(double)));
            size_t tmp = 0;
            LO_HIP(c, hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, c->d_ex_res, c->d_ex_sorted, static_cast<int>(n)));
            c->ex_sort_tmp_bytes = tmp;
            LO_HIP(c, hipMalloc(&c->d_ex_sort_tmp, tmp));
        }
        *n2 = 0;
        return LO_OK;
    }
    *n2 = static_cast<int>(n);
    return LO_OK;
}
// the iteration-0 scale of reference-exact mode (between the scan's first correspondence launch and its first PKO)
static void launch_exact_scale_any(lo_ctx* c, const KParams& P, int n2, hipStream_t s) {
    if (c->ex_merge && !c->ex_merge_presort) {
        launch_exact_scale_c(P, s);                          // counting sort + sums in one workgroup (<= 16384 points)
        return;
    }
    if (c->ex_merge) {
        // runs in the first half of d_ex_rank, the sorted keys in the second (kExactMaxPoints = 2 kExactMergeMax)
        launch_exact_scale_m(P, reinterpret_cast<const uint64_t*>(c->d_ex_rank),
                             reinterpret_cast<uint64_t*>(c->d_ex_rank) + kExactMergeMax, s);
        return;
    }
    if (n2 > 0) {
        launch_exact_scale(P, n2, c->d_ex_rank, s);
        return;
    }
    const int n = P.n;                                       // the bound (a device-filtered scan counts on the device)
    hipLaunchKernelGGL(k_exact_resid, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, P, c->d_ex_res);
    size_t tmp = c->ex_sort_tmp_bytes;
    (void)hipcub::DeviceRadixSort::SortKeys(c->d_ex_sort_tmp, tmp, c->d_ex_res, c->d_ex_sorted, n, 0,
                                            static_cast<int>(sizeof(double) * 8), s);
    launch_mwm_scale(P, c->d_ex_sorted, c->mwm, s);
}
static void launch_exact_iteration(lo_ctx* c, const KParams& P, const KParams& P0, int it, int n2, bool kd) {
    if (it == 0) launch_correspond_first(c, P0, kd, 0);   // (stage timing: the scan's first correspondence launch)
    else launch_correspond(c, P, 0, kd);
    if (it == 0) launch_exact_scale_any(c, P, n2, c->stream);
    launch_pko(c, P, it);
    hipLaunchKernelGGL(k_exact_terms, dim3(P.nb), dim3(kBlock), 0, c->stream, P);
    if (P.ex_ld) {                                           // large scan: 43 parallel sequential-sum reproductions
        launch_mw_sums(P.ex_terms, P.ex_ld, 43, P.n, P.n_dev, P.st, c->mw, P.ex_tot, nullptr, c->stream, LO_EXACT_FACTORED != 0);
        hipLaunchKernelGGL(k_exact_finish, dim3(1), dim3(64), 0, c->stream, P, it);
    } else {
        hipLaunchKernelGGL(k_exact_solve, dim3(1), dim3(512), 0, c->stream, P, it);   // kExactSolveThreads
    }
}

static int enqueue_optimize(lo_ctx* c, const float* d_pts, size_t n, const float T_init[12], const int* n_dev = nullptr) {
    const lo_config& g = c->cfg;
    std::memcpy(c->T_init, T_init, sizeof(float) * 12);
    c->last_n = n;
    c->last_pts = d_pts;
    c->last_ndev = n_dev;
    // reset the GN state (pose by kernel argument: no host staging buffer, scans can queue back to back)
    Pose12 T0;
    std::memcpy(T0.v, T_init, sizeof(float) * 12);
    // HIP events only for synchronous calls (gpu_ms): a marker packet costs ~5-7 us of device time per scan
    const bool timed = c->sync_call;
    c->last_timed = timed;
    if (timed) LO_HIP(c, hipEventRecord(c->ev0, c->stream));
    if (n == 0) {
        hipLaunchKernelGGL(k_init, dim3(1), dim3(64), 0, c->stream, c->d_st, T0, 1.0, g.robust_loss_delta);
    } else {
        const int rc = ensure_acc_part(c);
        if (rc != LO_OK) return rc;
        KParams P = make_params(c, d_pts, static_cast<int>(n));
        P.n_dev = n_dev;                                  // device-filtered scan: count read on the device
        KParams P0 = P;                                   // first k_correspond also resets the GN state
        P0.init = 1;
        std::memcpy(P0.T0, T_init, sizeof(float) * 12);
        std::memcpy(P.T0, T_init, sizeof(float) * 12);   // k_solve_correspond's pose before iteration 0
        // small scan with PKO: the solve of iteration it runs fused with the correspondence search of it + 1
        // (k_solve_correspond; KDTree: k_solve_knn, then k_knn_brute + k_plane), the last solve alone (k_solve_pick)
        const bool fused = spec_ok(P) && g.max_iterations <= LO_MAX_ITERS;
        int n2 = 0;
        if (c->exact) {
            const int rc3 = exact_prepare(c, P, n, &n2);
            if (rc3 != LO_OK) return rc3;
            P0.ex_terms = P.ex_terms;
            P0.scale_given = P.scale_given;
            if (c->ex_merge_presort) P0.presort = reinterpret_cast<uint64_t*>(c->d_ex_rank);
            if (!(fused && P.cand_rec && n2 > 0)) {
                // reference-exact GN loop without candidates (lo_exact.hip): correspondences, (iteration 0) sorted-order
                // scale, PKO, per-point fp32 terms, sequential sums + fp32 LDLT + SVD-projected update
                for (int it = 0; it < g.max_iterations; ++it) launch_exact_iteration(c, P, P0, it, n2, c->kd);
                LO_HIP(c, hipGetLastError());
                if (timed) LO_HIP(c, hipEventRecord(c->ev1, c->stream));
                c->pending = true;
                return LO_OK;
            }
            // small scans with PKO: the same launch sequence as the default mode, with the sorted-order scale after the
            // first correspondence launch and the PKO launch's candidates forming the reference's sequential sums
            P.exact_cand = P0.exact_cand = 1;
        }
        if (pipe_flagged(c)) {                            // an earlier scan's wait timed out: one stream from now on
            const int rc4 = pipe_recover(c);
            if (rc4 != LO_OK) return rc4;
        }
        if (fused && P.cand_rec && !c->kd && c->pipe && g.max_iterations > c->pipe_main) {
            // scan pipeline: iterations < pipe_main on the context stream, the rest on the tail stream behind a
            // device-side wait for the main part; k_wait_final then holds the context stream until the scan's result
            // is final
            const int rc2 = pipe_alloc(c);
            if (rc2 != LO_OK) return rc2;
            if (++c->pipe_seq == 0) c->pipe_seq = 1;      // 0 is the fence word's reset value, never a scan's number
            const uint32_t seq = c->pipe_seq;
            P.fin = P0.fin = c->d_fin;
            P.seq = P0.seq = seq;
            KParams Pt = P;                               // tail launches: leave once scan seq is final (the
            Pt.tail = 1;                                  // DevState may already be the next scan's)
            KParams Ph = P;                               // the main part's last pick signals the tail (signal_main)
            Ph.hold = 1;
            // host submission order main -> tail -> k_wait_final: every device-side wait depends only on work
            // submitted before it (deadlock-free even if the two streams share a hardware queue)
            launch_correspond_first(c, P0, false);
            if (c->exact) launch_exact_scale_any(c, P, n2, c->stream);
            for (int it = 0; it < g.max_iterations; ++it) {
                const bool tail = it >= c->pipe_main;
                if (it == c->pipe_main)                   // bound 0: the test hook's forced timeout
                    hipLaunchKernelGGL(k_wait_seq, dim3(1), dim3(kWave), 0, c->s_tail, c->d_fin, seq, c->d_st, c->d_hbroken,
                                       (c->pipe_fail_at != 0 && seq == c->pipe_fail_at) ? 0ull : c->pipe_bound);
                const hipStream_t s = tail ? c->s_tail : c->stream;
                const KParams& Pi = tail ? Pt : (it + 1 == c->pipe_main ? Ph : P);
                launch_pko_spec(c, Pi, it, s);
                if (it + 1 < g.max_iterations) hipLaunchKernelGGL(k_pick_correspond, dim3(P.nb), dim3(kBlock), 0, s, Pi, it);
                else hipLaunchKernelGGL(k_pick, dim3(1), dim3(kBlock), 0, s, Pi, it);
            }
            hipLaunchKernelGGL(k_wait_final, dim3(1), dim3(kWave), 0, c->stream, c->d_fin, seq, c->d_st, c->d_hbroken,
                               c->pipe_bound);
            LO_HIP(c, hipGetLastError());
            if (timed) LO_HIP(c, hipEventRecord(c->ev1, c->stream));
            c->pending = true;
            return LO_OK;
        }
        for (int it = 0; it < g.max_iterations; ++it) {
            if (!fused) {
                if (it == 0) launch_correspond_first(c, P0, c->kd);
                else launch_correspond(c, P, 0, c->kd);
                launch_gn_tail(c, P, it);
                continue;
            }
            if (it == 0) {
                launch_correspond_first(c, P0, c->kd);
                if (c->exact) launch_exact_scale_any(c, P, n2, c->stream);
            }
            launch_pko_spec(c, P, it);
            if (it + 1 < g.max_iterations && !c->kd) {
                if (P.cand_rec) hipLaunchKernelGGL(k_pick_correspond, dim3(P.nb), dim3(kBlock), 0, c->stream, P, it);
                else hipLaunchKernelGGL(k_solve_correspond, dim3(P.nb), dim3(kBlock), 0, c->stream, P, it);
            } else if (it + 1 < g.max_iterations) {
                launch_pick_knn(c, P, it);
            } else if (P.cand_rec) {
                hipLaunchKernelGGL(k_pick, dim3(1), dim3(kBlock), 0, c->stream, P, it);
            } else {
                hipLaunchKernelGGL(k_solve_pick, dim3(1), dim3(kBlock), 0, c->stream, P, it);
            }
        }
        LO_HIP(c, hipGetLastError());
    }
    if (timed) LO_HIP(c, hipEventRecord(c->ev1, c->stream));
    c->pending = true;
    return LO_OK;
}

int lo_icp_optimize_async(lo_ctx* c, const float* d_pts, size_t n, const float T_init[12]) {
    if (!c || !T_init || (n > 0 && !d_pts)) return LO_ERR_ARG;
    if (n > static_cast<size_t>(c->cfg.max_points)) { c->err = "n exceeds max_points"; return LO_ERR_CAPACITY; }
    LO_HIP(c, hipSetDevice(c->device));
    c->last_dev_count = false;
    c->nf_valid = false;
    return enqueue_optimize(c, d_pts, n, T_init);
}

int lo_icp_result(lo_ctx* c, float T_out[12], lo_iter_log* logs, lo_stats* st) {
    if (!c) return LO_ERR_ARG;
    if (!c->pending) { c->err = "no optimize in flight"; return LO_ERR_STATE; }
    // state header + the executed iterations' logs only
    const size_t bytes = offsetof(DevState, logs) + sizeof(lo_iter_log) * static_cast<size_t>(c->cfg.max_iterations);
    LO_HIP(c, hipMemcpyAsync(c->h_st, c->d_st, bytes, hipMemcpyDeviceToHost, c->stream));
    // a device-filtered scan: its count comes back in the same sync (lo_filtered_points(ctx, NULL, 0) then reads it
    // without another round trip -- the frame loop asks for it every frame)
    c->nf_valid = c->last_dev_count && c->vf.n_out;
    if (c->nf_valid) LO_HIP(c, hipMemcpyAsync(c->h_nf, c->vf.n_out, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    LO_HIP(c, hipStreamSynchronize(c->stream));
    c->pending = false;
    const DevState* hs = c->h_st;
    int status = c->last_n == 0 ? LO_INSUFFICIENT : hs->status;
    if (status == LO_ERR_PIPELINE) {
        // this scan's pipeline wait timed out: pipeline off, then the same scan again on one stream (its points are
        // still the caller's until this call returns)
        int rc = pipe_recover(c);
        if (rc != LO_OK) return rc;
        float T0[12];
        std::memcpy(T0, c->T_init, sizeof(T0));
        const bool timed = c->sync_call;
        rc = enqueue_optimize(c, c->last_pts, c->last_n, T0, c->last_ndev);
        c->sync_call = timed;
        if (rc != LO_OK) return rc;
        LO_HIP(c, hipMemcpyAsync(c->h_st, c->d_st, bytes, hipMemcpyDeviceToHost, c->stream));
        LO_HIP(c, hipStreamSynchronize(c->stream));
        c->pending = false;
        ++c->pipe_reruns;
        status = hs->status;
    }
    if (c->kd && c->grid_dev && !c->grid.has_order && hs->kd_tie && c->last_n > 0) {
        // a deciding distance tie was ranked by index (a device-built grid has no kd visit order): the order built on
        // the host from the grid's own points, then the same scan again (its points are still the caller's)
        int rc = grid_add_order(c);
        if (rc != LO_OK) return rc;
        float T0[12];
        std::memcpy(T0, c->T_init, sizeof(T0));
        const bool timed = c->sync_call;
        rc = enqueue_optimize(c, c->last_pts, c->last_n, T0, c->last_ndev);
        c->sync_call = timed;
        if (rc != LO_OK) return rc;
        LO_HIP(c, hipMemcpyAsync(c->h_st, c->d_st, bytes, hipMemcpyDeviceToHost, c->stream));
        LO_HIP(c, hipStreamSynchronize(c->stream));
        c->pending = false;
        ++c->kd_reruns;
        status = hs->status;
    }
    const int iters = hs->iter;
    if (T_out) {
        if (status == LO_OK) std::memcpy(T_out, hs->pose, sizeof(float) * 12);
        else std::memcpy(T_out, c->T_init, sizeof(float) * 12);   // optimized_transform = initial (:266, :301)
    }
    if (logs) for (int i = 0; i < iters && i < c->cfg.max_iterations; ++i) logs[i] = hs->logs[i];
    if (st) {
        st->iterations = iters;
        st->n_corr = hs->n_corr;
        st->status = status;
        st->converged = status == LO_OK ? 1 : 0;
        st->initial_cost = iters > 0 ? hs->logs[0].cost : 0.0;
        st->final_cost = iters > 0 ? hs->logs[iters - 1].cost : 0.0;
        float ms = -1.0f;                                  // -1: an async call (not timed)
        if (c->last_timed && hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess) ms = -1.0f;
        st->gpu_ms = ms;
    }
    return status;
}

int lo_sync(lo_ctx* c) {
    if (!c) return LO_ERR_ARG;
    LO_HIP(c, sync_all(c));
    return LO_OK;
}

int lo_icp_optimize(lo_ctx* c, const float* pts, size_t n, const float T_init[12], float T_out[12],
                    lo_iter_log* logs, lo_stats* st) {
    if (!c || !T_init || !T_out || (n > 0 && !pts)) return LO_ERR_ARG;
    if (n > static_cast<size_t>(c->cfg.max_points)) { c->err = "n exceeds max_points"; return LO_ERR_CAPACITY; }
    LO_HIP(c, hipSetDevice(c->device));
    if (n > 0) LO_HIP(c, hipMemcpyAsync(c->d_pts, pts, n * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    c->last_dev_count = false;
    c->nf_valid = false;
    c->sync_call = true;
    int rc = enqueue_optimize(c, c->d_pts, n, T_init);
    c->sync_call = false;
    if (rc != LO_OK) return rc;
    return lo_icp_result(c, T_out, logs, st);
}

// ---------------------------------------------------------------- loop-closure ICP
// IterativeClosestPointOptimizer::optimize_loop (:40-251) + find_correspondences_loop (:465-585): the KDTree
// correspondence kernels against the matched keyframe's local map (its own grid, so the context's odometry map
// is left alone), no distance gate, up to 100 GN iterations enqueued kLoopChunk at a time between convergence
// checks, then the 1-NN inlier ratio (k_inlier) once converged.
static constexpr int kLoopMaxIters = 100;                // :74
static constexpr int kLoopChunk = 4;
static constexpr int kLoopMinPerCell = 4;                // the matched cloud's grid: >= 4 points per occupied cell

int lo_icp_optimize_loop(lo_ctx* c, const float* curr, size_t n_curr, const float T_curr[12], const float* matched,
                         size_t n_matched, const float T_matched[12], float T_rel_out[12], float* inlier_ratio,
                         lo_iter_log* logs, lo_stats* st) {
    if (!c || !T_curr || !T_matched || !T_rel_out || !inlier_ratio || (n_curr > 0 && !curr) || (n_matched > 0 && !matched))
        return LO_ERR_ARG;
    if (n_curr > static_cast<size_t>(c->cfg.max_points)) { c->err = "n_curr exceeds max_points"; return LO_ERR_CAPACITY; }
    LO_HIP(c, hipSetDevice(c->device));
    int rc = kd_alloc(c);
    if (rc != LO_OK) return rc;
    // local map of the matched keyframe: its feature cloud in the world (transform_point_cloud, :60-64)
    const lo::SE3f Tm = lo::se3_from12(T_matched);
    std::vector<float> lmap(3 * std::max<size_t>(n_matched, 1));
    if (n_matched > 0) lo::transform_points(Tm, matched, n_matched, lmap.data());
    // the matched cloud's grid first without the kd visit order (building it is ~0.3 ms of host work per call and
    // it only ranks exact distance ties that decide a query's five neighbours or their order, which keyframe
    // centroids rarely produce); a solve that met one is rerun with the order below
    bool with_order = false;
    const bool all = n_matched <= static_cast<size_t>(kKnnAllMax);     // (the clouds' pinned upload, curr included)
    rc = all ? all_pairs_upload(c, c->lgrid, lmap.data(), n_matched, curr, n_curr)
             : grid_build(c, c->lgrid, lmap.data(), n_matched, with_order, kLoopMinPerCell);
    if (rc != LO_OK) return rc;
retry:
    if (st) { std::memset(st, 0, sizeof(*st)); st->status = LO_INSUFFICIENT; }
    if (n_curr == 0 || n_matched == 0) return LO_INSUFFICIENT;       // empty clouds: 0 correspondences (:477-483)
    if ((rc = ensure_acc_part(c)) != LO_OK) return rc;
    if (!c->lgrid.all) LO_HIP(c, hipMemcpyAsync(c->d_pts, curr, n_curr * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    KParams P = make_params(c, c->d_pts, static_cast<int>(n_curr));
    set_kd_params(c, P, c->lgrid);
    P.loop = 1;
    std::memcpy(P.Tm, T_matched, sizeof(float) * 12);
    // T_lw_last = T_wl_last.inverse() (:509): the rigid inverse [R^T | -R^T t], evaluated in fp64 and rounded
    for (int r = 0; r < 3; ++r) {
        double tr = 0.0;
        for (int k = 0; k < 3; ++k) {
            P.Tlw[4 * r + k] = T_matched[4 * k + r];
            tr -= static_cast<double>(T_matched[4 * k + r]) * static_cast<double>(T_matched[4 * k + 3]);
        }
        P.Tlw[4 * r + 3] = static_cast<float>(tr);
    }
    int n2 = 0;
    if (c->exact && (rc = exact_prepare(c, P, n_curr, &n2)) != LO_OK) return rc;
    KParams P0 = P;
    P0.init = 1;
    if (c->exact && c->ex_merge_presort) P0.presort = reinterpret_cast<uint64_t*>(c->d_ex_rank);
    std::memcpy(P0.T0, T_curr, sizeof(float) * 12);
    // small clouds with PKO: the odometry path's launch sequence (candidates solved in the PKO launch, k_pick_knn
    // taking the selected one fused with the next kNN search); reference-exact mode as there
    const bool cand = spec_ok(P) && P.cand_rec && (!c->exact || n2 > 0);
    if (cand && c->exact) { P.exact_cand = P0.exact_cand = 1; P0.ex_terms = P.ex_terms; }
    const dim3 blk(kBlock);
    LO_HIP(c, hipEventRecord(c->ev0, c->stream));
    const size_t head = offsetof(DevState, logs);
    for (int it = 0; it < kLoopMaxIters;) {
        for (int k = 0; k < kLoopChunk && it < kLoopMaxIters; ++k, ++it) {
            if (cand) {
                if (it == 0) {
                    launch_correspond(c, P0, 1, true);
                    if (c->exact) launch_exact_scale_any(c, P, n2, c->stream);
                }
                launch_pko_spec(c, P, it);
                if (it + 1 < kLoopMaxIters) launch_pick_knn(c, P, it);
                else hipLaunchKernelGGL(k_pick, dim3(1), blk, 0, c->stream, P, it);
                continue;
            }
            if (c->exact) {
                launch_exact_iteration(c, P, P0, it, n2, true);
                continue;
            }
            launch_correspond(c, it == 0 ? P0 : P, it == 0 ? 1 : 0, true);
            launch_gn_tail(c, P, it);
        }
        LO_HIP(c, hipGetLastError());
        LO_HIP(c, hipMemcpyAsync(c->h_st, c->d_st, head, hipMemcpyDeviceToHost, c->stream));
        LO_HIP(c, hipStreamSynchronize(c->stream));
        if (c->h_st->done) break;                                 // converged, or too few correspondences
    }
    const bool converged = c->h_st->done && c->h_st->status == LO_OK;
    if (converged && P.kd_all) hipLaunchKernelGGL(k_inlier_all, all_grid(P), dim3(kAllThreads), all_lds(P), c->stream, P);
    else if (converged) hipLaunchKernelGGL(k_inlier, dim3(P.nb), blk, 0, c->stream, P);
    LO_HIP(c, hipGetLastError());
    LO_HIP(c, hipEventRecord(c->ev1, c->stream));
    const size_t bytes = head + sizeof(lo_iter_log) * static_cast<size_t>(LO_MAX_ITERS);
    LO_HIP(c, hipMemcpyAsync(c->h_st, c->d_st, bytes, hipMemcpyDeviceToHost, c->stream));
    LO_HIP(c, hipStreamSynchronize(c->stream));
    if (c->h_st->kd_tie && !with_order) {               // a deciding tie was ranked by index: redo with the order
        with_order = true;
        ++c->loop_reruns;
        rc = grid_build(c, c->lgrid, lmap.data(), n_matched, true, kLoopMinPerCell);
        if (rc != LO_OK) return rc;
        goto retry;
    }
    const DevState* hs = c->h_st;
    bool success = false;
    if (converged) {
        // optimized_relative_transform = curr.pose^-1 * optimized_curr_pose (:240), set on convergence
        const lo::SE3f rel = lo::se3_mul(lo::se3_inv(lo::se3_from12(T_curr)), lo::se3_from12(hs->pose));
        lo::se3_to12(rel, T_rel_out);
        *inlier_ratio = static_cast<float>(static_cast<int>(hs->inliers)) / static_cast<float>(static_cast<int>(n_curr));
        success = !(*inlier_ratio < 0.5f);                            // :244-246
    }
    const int iters = hs->iter;
    if (logs) for (int i = 0; i < iters && i < LO_MAX_ITERS; ++i) logs[i] = hs->logs[i];
    const int status = success ? LO_OK : LO_INSUFFICIENT;
    if (st) {
        st->iterations = iters;
        st->n_corr = hs->n_corr;
        st->status = status;
        st->converged = converged ? 1 : 0;
        const int last = std::min(iters, LO_MAX_ITERS) - 1;
        st->initial_cost = iters > 0 ? hs->logs[0].cost : 0.0;
        st->final_cost = last >= 0 ? hs->logs[last].cost : 0.0;
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess) ms = -1.0f;
        st->gpu_ms = ms;
    }
    c->pending = false;
    return status;
}

// ---------------------------------------------------------------- device preprocessing + optimize
static int stage_raw(lo_ctx* c, const float* raw, size_t n_raw) {
    if (n_raw > c->raw_cap) {
        if (c->d_raw) LO_HIP(c, hipFree(c->d_raw));
        c->d_raw = nullptr;
        LO_HIP(c, hipMalloc(&c->d_raw, n_raw * 3 * sizeof(float)));
        c->raw_cap = n_raw;
    }
    if (n_raw > 0) LO_HIP(c, hipMemcpyAsync(c->d_raw, raw, n_raw * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    return LO_OK;
}

static int check_raw_args(lo_ctx* c, size_t n_raw, int stride, float voxel) {
    if (stride < 1 || !(voxel > 0.0f)) { c->err = "stride must be >= 1 and voxel_size > 0"; return LO_ERR_ARG; }
    const size_t m = (n_raw + stride - 1) / stride;
    if (m > static_cast<size_t>(c->cfg.max_points)) { c->err = "ceil(n_raw / stride) exceeds max_points"; return LO_ERR_CAPACITY; }
    return LO_OK;
}

int lo_icp_optimize_raw_async(lo_ctx* c, const float* d_raw, size_t n_raw, int stride, float voxel_size,
                              const float T_init[12]) {
    if (!c || !T_init || (n_raw > 0 && !d_raw)) return LO_ERR_ARG;
    int rc = check_raw_args(c, n_raw, stride, voxel_size);
    if (rc != LO_OK) return rc;
    LO_HIP(c, hipSetDevice(c->device));
    int m = 0;
    LO_HIP(c, vf_enqueue(c->vf, d_raw, n_raw, stride, voxel_size, c->d_pts, c->stream, m));
    c->last_dev_count = true;
    c->nf_valid = false;
    return enqueue_optimize(c, c->d_pts, static_cast<size_t>(m), T_init, c->vf.n_out);
}

// A host scan in pinned memory (lo_host_alloc, hipHostMalloc, hipHostRegister): the device address that aliases it,
// so the filter reads the sampled points over the bus directly instead of a staging copy of the whole scan.
static const float* pinned_alias(const float* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return nullptr; }   // pageable
    if (a.type != hipMemoryTypeHost || !a.devicePointer || !a.hostPointer) return nullptr;
    return reinterpret_cast<const float*>(static_cast<const char*>(a.devicePointer) +
                                          (reinterpret_cast<const char*>(p) - static_cast<const char*>(a.hostPointer)));
}

void* lo_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void lo_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int lo_icp_optimize_raw(lo_ctx* c, const float* raw, size_t n_raw, int stride, float voxel_size, const float T_init[12],
                        float T_out[12], lo_iter_log* logs, lo_stats* st) {
    if (!c || !T_init || !T_out || (n_raw > 0 && !raw)) return LO_ERR_ARG;
    int rc = check_raw_args(c, n_raw, stride, voxel_size);
    if (rc != LO_OK) return rc;
    LO_HIP(c, hipSetDevice(c->device));
    const float* src = n_raw > 0 ? pinned_alias(raw) : nullptr;
    if (!src) {                                          // pageable: stage the scan in device memory
        rc = stage_raw(c, raw, n_raw);
        if (rc != LO_OK) return rc;
        src = c->d_raw;
    }
    c->sync_call = true;
    rc = lo_icp_optimize_raw_async(c, src, n_raw, stride, voxel_size, T_init);
    c->sync_call = false;
    if (rc != LO_OK) return rc;
    return lo_icp_result(c, T_out, logs, st);
}

long long lo_filtered_points(lo_ctx* c, float* out, size_t cap) {
    if (!c) return LO_ERR_ARG;
    if (!c->last_dev_count || !c->vf.n_out) { c->err = "no device-filtered scan"; return LO_ERR_STATE; }
    if (!out && c->nf_valid && !c->pending) return *c->h_nf;   // read back with the scan's result (lo_icp_result)
    LO_HIP(c, hipSetDevice(c->device));
    int n = 0;
    LO_HIP(c, hipMemcpyAsync(&n, c->vf.n_out, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    LO_HIP(c, hipStreamSynchronize(c->stream));
    if (out && n > 0) {
        const size_t k = std::min<size_t>(static_cast<size_t>(n), cap);
        LO_HIP(c, hipMemcpy(out, c->d_pts, k * 3 * sizeof(float), hipMemcpyDeviceToHost));
    }
    return n;
}

long long lo_voxel_filter_gpu(lo_ctx* c, const float* raw, size_t n_raw, float voxel_size, int stride, float* out,
                              size_t out_cap) {
    if (!c || (n_raw > 0 && !raw)) return LO_ERR_ARG;
    int rc = check_raw_args(c, n_raw, stride, voxel_size);
    if (rc != LO_OK) return rc;
    LO_HIP(c, hipSetDevice(c->device));
    rc = stage_raw(c, raw, n_raw);
    if (rc != LO_OK) return rc;
    int m = 0;
    LO_HIP(c, vf_enqueue(c->vf, c->d_raw, n_raw, stride, voxel_size, c->d_pts, c->stream, m));
    c->last_dev_count = true;
    c->nf_valid = false;
    return lo_filtered_points(c, out, out_cap);
}

// ---------------------------------------------------------------- parity entry points
static int ensure_res(lo_ctx* c, size_t n) {
    if (c->res_cap >= n && c->d_res) return LO_OK;
    if (c->d_res) { LO_HIP(c, hipFree(c->d_res)); c->d_res = nullptr; }
    if (c->d_u8) { LO_HIP(c, hipFree(c->d_u8)); c->d_u8 = nullptr; }
    const size_t cap = std::max<size_t>(n, 256);
    LO_HIP(c, hipMalloc(&c->d_res, cap * sizeof(double)));
    LO_HIP(c, hipMalloc(&c->d_u8, cap));
    c->res_cap = cap;
    return LO_OK;
}

static int reset_state(lo_ctx* c, const float T[12], double scale, double alpha) {
    Pose12 T0;
    std::memcpy(T0.v, T, sizeof(float) * 12);
    hipLaunchKernelGGL(k_init, dim3(1), dim3(64), 0, c->stream, c->d_st, T0, scale, alpha);
    LO_HIP(c, hipGetLastError());
    return LO_OK;
}

int lo_find_correspondences(lo_ctx* c, const float* pts, size_t n, const float T[12], uint8_t* valid, double* residual) {
    if (!c || !T || (n > 0 && (!pts || !valid || !residual))) return LO_ERR_ARG;
    if (n > static_cast<size_t>(c->cfg.max_points)) { c->err = "n exceeds max_points"; return LO_ERR_CAPACITY; }
    if (n == 0) return 0;
    LO_HIP(c, hipSetDevice(c->device));
    int rc = ensure_res(c, n);
    if (rc != LO_OK) return rc;
    rc = reset_state(c, T, 1.0, 0.1);
    if (rc != LO_OK) return rc;
    LO_HIP(c, hipMemcpyAsync(c->d_pts, pts, n * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    KParams P = make_params(c, c->d_pts, static_cast<int>(n));
    P.res_dbg = c->d_res;
    launch_correspond(c, P, 1, c->kd);
    LO_HIP(c, hipGetLastError());
    std::vector<int32_t> slots(n);
    LO_HIP(c, hipMemcpyAsync(slots.data(), c->d_slot, n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    LO_HIP(c, hipMemcpyAsync(residual, c->d_res, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    LO_HIP(c, hipStreamSynchronize(c->stream));
    int cnt = 0;
    for (size_t i = 0; i < n; ++i) { valid[i] = slots[i] >= 0 ? 1 : 0; cnt += valid[i]; }
    return cnt;
}

int lo_knn_search(lo_ctx* c, const float* q, size_t n, int32_t* idx, float* dist) {
    if (!c || (n > 0 && (!q || !idx || !dist))) return LO_ERR_ARG;
    if (!c->kd) { c->err = "lo_knn_search needs use_surfel_correspondence = 0"; return LO_ERR_STATE; }
    if (n > static_cast<size_t>(c->cfg.max_points)) { c->err = "n exceeds max_points"; return LO_ERR_CAPACITY; }
    if (n == 0) return 0;
    LO_HIP(c, hipSetDevice(c->device));
    const float I[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};       // Matrix4f * (x, y, z, 1) is exact at I
    int rc = reset_state(c, I, 1.0, 0.1);
    if (rc != LO_OK) return rc;
    LO_HIP(c, hipMemcpyAsync(c->d_pts, q, n * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    KParams P = make_params(c, c->d_pts, static_cast<int>(n));
    KParams Pn = P;
    Pn.init = 0;
    hipLaunchKernelGGL(k_knn, dim3((n * kKnnGroup + kBlock - 1) / kBlock), dim3(kBlock), 0, c->stream, P);
    launch_brute(c, Pn);
    hipLaunchKernelGGL(k_knn_reset, dim3(1), dim3(64), 0, c->stream, Pn);
    LO_HIP(c, hipGetLastError());
    std::vector<int32_t> nb(5 * n);
    std::vector<float4> mp(static_cast<size_t>(std::max(c->grid.m, 1)));
    LO_HIP(c, hipMemcpyAsync(nb.data(), c->d_kd_nbr, nb.size() * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    if (c->grid.m > 0)
        LO_HIP(c, hipMemcpyAsync(mp.data(), c->grid.d_pts, c->grid.m * sizeof(float4), hipMemcpyDeviceToHost, c->stream));
    LO_HIP(c, hipStreamSynchronize(c->stream));
    int cnt = 0;
    for (size_t i = 0; i < n; ++i) {
        const bool ok = nb[5 * i] >= 0;
        cnt += ok ? 1 : 0;
        for (int k = 0; k < 5; ++k) {
            if (!ok) { idx[5 * i + k] = -1; dist[5 * i + k] = INFINITY; continue; }
            const float4 v = mp[nb[5 * i + k]];
            int32_t id;
            std::memcpy(&id, &v.w, sizeof(id));
            const float dx = q[3 * i] - v.x, dy = q[3 * i + 1] - v.y, dz = q[3 * i + 2] - v.z;
            idx[5 * i + k] = id;
            dist[5 * i + k] = (dx * dx + dy * dy) + dz * dz;
        }
    }
    return cnt;
}

double lo_pko_scale_factor(lo_ctx* c, const double* residuals, size_t n, double* gmm_out) {
    if (!c || (n > 0 && !residuals)) return NAN;
    if (n == 0) return 1.0;                                  // calculate_scale_factor, empty input (:66-69)
    if (n > static_cast<size_t>(c->cfg.max_points)) { c->err = "n exceeds max_points"; return NAN; }
    if (hipSetDevice(c->device) != hipSuccess) return NAN;
    if (ensure_res(c, n) != LO_OK) return NAN;
    const float I[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    if (reset_state(c, I, 1.0, 0.1) != LO_OK) return NAN;
    if (hipMemcpyAsync(c->d_res, residuals, n * sizeof(double), hipMemcpyHostToDevice, c->stream) != hipSuccess) return NAN;
    KParams P = make_params(c, c->d_pts, static_cast<int>(n));
    P.direct_res = c->d_res;
    P.use_pko = 1;
    launch_pko(c, P, 0);
    hipLaunchKernelGGL(k_pko_finish, dim3(1), dim3(64), 0, c->stream, P);
    if (hipGetLastError() != hipSuccess) return NAN;
    if (hipMemcpyAsync(c->h_st, c->d_st, sizeof(DevState), hipMemcpyDeviceToHost, c->stream) != hipSuccess) return NAN;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return NAN;
    if (gmm_out) for (int j = 0; j < 3 * c->cfg.gmm_components; ++j) gmm_out[j] = c->h_st->gmm_out[j];
    return c->h_st->alpha;
}

int lo_build_normal_equations(lo_ctx* c, const float* pts, size_t n, const float T[12], double scale, double delta,
                              double H[36], double g[6], double* cost) {
    if (!c || !T || !H || !g || !cost || (n > 0 && !pts)) return LO_ERR_ARG;
    if (n > static_cast<size_t>(c->cfg.max_points)) { c->err = "n exceeds max_points"; return LO_ERR_CAPACITY; }
    if (n == 0) { std::memset(H, 0, 36 * sizeof(double)); std::memset(g, 0, 6 * sizeof(double)); *cost = 0; return 0; }
    LO_HIP(c, hipSetDevice(c->device));
    int rc = reset_state(c, T, scale, delta);
    if (rc != LO_OK) return rc;
    LO_HIP(c, hipMemcpyAsync(c->d_pts, pts, n * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    KParams P = make_params(c, c->d_pts, static_cast<int>(n));
    P.alpha_given = 1;
    launch_correspond(c, P, 0, c->kd);
    if (P.nb_acc <= kFuseMaxBlocks) {
        hipLaunchKernelGGL(k_accumulate, dim3(P.nb_acc), dim3(kBlock), 0, c->stream, P, 0, 2);
    } else {
        hipLaunchKernelGGL(k_accumulate, dim3(P.nb_acc), dim3(kBlock), 0, c->stream, P, 0, 0);
        hipLaunchKernelGGL(k_solve, dim3(1), dim3(kSolveThreads), 0, c->stream, P, 0, 1);
    }
    LO_HIP(c, hipGetLastError());
    std::vector<int32_t> cnt(P.nb);
    LO_HIP(c, hipMemcpyAsync(cnt.data(), c->d_blk_cnt, P.nb * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    LO_HIP(c, hipMemcpyAsync(c->h_st, c->d_st, sizeof(DevState), hipMemcpyDeviceToHost, c->stream));
    LO_HIP(c, hipStreamSynchronize(c->stream));
    for (int q = 0; q < 36; ++q) H[q] = c->h_st->H_out[q];
    for (int j = 0; j < 6; ++j) g[j] = c->h_st->g_out[j];
    *cost = c->h_st->cost_out;
    int total = 0;
    for (int v : cnt) total += v;
    return total;
}

int lo_pko_sample_indices(lo_ctx* c, size_t n, int32_t* out) {
    if (!c || !out) return LO_ERR_ARG;
    if (n > static_cast<size_t>(c->cfg.max_points)) { c->err = "n exceeds max_points"; return LO_ERR_CAPACITY; }
    const int k = static_cast<int>(std::min<size_t>(n, static_cast<size_t>(c->cfg.gmm_sample_size)));
    for (int s = 0; s < k; ++s) out[s] = pko_sample_host(c->tables, static_cast<int>(n), s);
    return k;
}

// start stamps ~0, end stamps 0, in every launch's record (kStageEvents + 1 records)
static int reset_spans(lo_ctx* c) {
    const size_t words = static_cast<size_t>(kSpanWords) * (kStageEvents + 1);
    if (!c->d_span) LO_HIP(c, hipMalloc(&c->d_span, words * sizeof(unsigned long long)));
    std::vector<unsigned long long> h(words, 0ull);
    for (size_t r = 0; r < words; r += kSpanWords)
        for (int k = 0; k < kSpanStarts; ++k) h[r + k] = ~0ull;
    LO_HIP(c, hipMemcpyAsync(c->d_span, h.data(), h.size() * sizeof(unsigned long long), hipMemcpyHostToDevice, c->stream));
    LO_HIP(c, hipStreamSynchronize(c->stream));
    return LO_OK;
}

// a launch's span record: the latest end stamp minus the earliest start stamp (0 if it did not run)
static unsigned long long span_of(const unsigned long long* r) {
    unsigned long long s = ~0ull, e = 0;
    for (int k = 0; k < kSpanStarts; ++k) s = std::min(s, r[k]);
    for (int k = 0; k < kSpanEnds; ++k) e = std::max(e, r[kSpanStarts + k]);
    return e > s ? e - s : 0ull;
}

int lo_set_stage_timing(lo_ctx* c, int enable) {
    if (!c) return LO_ERR_ARG;
    if (enable && c->st_ev.empty()) {
        c->st_ev.resize(2 * kStageEvents, nullptr);
        for (hipEvent_t& e : c->st_ev) LO_HIP(c, hipEventCreate(&e));
    }
    if (enable) {
        LO_HIP(c, hipSetDevice(c->device));
        const int rc = reset_spans(c);
        if (rc != LO_OK) return rc;
    }
    c->stage_timing = enable != 0;
    c->st_n = 0;
    return LO_OK;
}

int lo_stage_span(lo_ctx* c, double* avg_us, int* count) {
    if (!c || !avg_us) return LO_ERR_ARG;
    *avg_us = 0.0;
    if (count) *count = 0;
    if (!c->d_span || c->st_n == 0) return LO_OK;
    LO_HIP(c, hipSetDevice(c->device));
    LO_HIP(c, hipStreamSynchronize(c->stream));
    std::vector<unsigned long long> h(static_cast<size_t>(kSpanWords) * c->st_n);
    LO_HIP(c, hipMemcpy(h.data(), c->d_span, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    double tot = 0.0;
    int k = 0;
    for (int i = 0; i < c->st_n; ++i) {
        const unsigned long long d = span_of(h.data() + static_cast<size_t>(kSpanWords) * i);
        if (d) { tot += static_cast<double>(d); ++k; }
    }
    *avg_us = k ? tot / k * 0.01 : 0.0;                  // s_memrealtime: 100 MHz
    if (count) *count = k;
    return LO_OK;
}

int lo_stage_time(lo_ctx* c, double* avg_us, int* count) {
    if (!c || !avg_us) return LO_ERR_ARG;
    LO_HIP(c, hipStreamSynchronize(c->stream));
    double tot = 0.0;
    for (int i = 0; i < c->st_n; ++i) {
        float ms = 0.0f;
        LO_HIP(c, hipEventElapsedTime(&ms, c->st_ev[2 * i], c->st_ev[2 * i + 1]));
        tot += ms;
    }
    *avg_us = c->st_n > 0 ? tot * 1e3 / c->st_n : 0.0;
    if (count) *count = c->st_n;
    return LO_OK;
}

int lo_pko_em_stats(lo_ctx* c, unsigned long long out[3], int reset) {
    if (!c || !out) return LO_ERR_ARG;
    LO_HIP(c, hipSetDevice(c->device));
    LO_HIP(c, sync_all(c));
    LO_HIP(c, hipMemcpy(out, reinterpret_cast<const char*>(c->d_st) + offsetof(DevState, em_stat),
                        3 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    if (reset)
        LO_HIP(c, hipMemset(reinterpret_cast<char*>(c->d_st) + offsetof(DevState, em_stat), 0, 3 * sizeof(unsigned long long)));
    return LO_OK;
}

int lo_set_exact(lo_ctx* c, int enable) {
    if (!c) return LO_ERR_ARG;
    c->exact = enable != 0;
    return LO_OK;
}

int lo_set_pko_groups(lo_ctx* c, int groups) {
    if (!c || groups < 0) return LO_ERR_ARG;
    c->pko_groups = groups;
    return LO_OK;
}

int lo_pipeline_status(lo_ctx* c, int out[4]) {
    if (!c || !out) return LO_ERR_ARG;
    out[0] = c->pipe ? 1 : 0;
    out[1] = c->pipe_main;
    out[2] = static_cast<int>(c->pipe_timeouts);
    out[3] = static_cast<int>(c->pipe_reruns);
    return LO_OK;
}

int lo_set_pipeline(lo_ctx* c, int enable, int main_iterations) {
    if (!c || main_iterations < 0) return LO_ERR_ARG;
    c->pipe = enable != 0;
    if (main_iterations > 0) c->pipe_main = main_iterations;
    return LO_OK;
}

int lo_set_stream(lo_ctx* c, void* stream) {
    if (!c) return LO_ERR_ARG;
    LO_HIP(c, hipSetDevice(c->device));
    LO_HIP(c, sync_all(c));
    if (c->own_stream) { LO_HIP(c, hipStreamDestroy(c->stream)); c->own_stream = false; }
    if (stream) c->stream = static_cast<hipStream_t>(stream);
    else { LO_HIP(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)); c->own_stream = true; }
    return LO_OK;
}

int lo_icp_export_pose(lo_ctx* c, float* d_out16) {
    if (!c || !d_out16) return LO_ERR_ARG;
    hipLaunchKernelGGL(k_export_pose, dim3(1), dim3(64), 0, c->stream, c->d_st, d_out16);
    LO_HIP(c, hipGetLastError());
    return LO_OK;
}

int lo_bench_kernel(lo_ctx* c, const float* d_pts, size_t n, const float T[12], double scale, double alpha,
                    int kernel_id, int reps, float* avg_ms) {
    if (!c || !d_pts || !T || !avg_ms || n == 0 || reps < 1 || kernel_id < 0 || kernel_id > 5) return LO_ERR_ARG;
    if (kernel_id == 5 && c->kd) { c->err = "kernel 5: surfel correspondence only"; return LO_ERR_STATE; }
    if (n > static_cast<size_t>(c->cfg.max_points)) { c->err = "n exceeds max_points"; return LO_ERR_CAPACITY; }
    LO_HIP(c, hipSetDevice(c->device));
    int rc = reset_state(c, T, scale, alpha);
    if (rc != LO_OK) return rc;
    if ((rc = ensure_acc_part(c)) != LO_OK) return rc;
    KParams P = make_params(c, d_pts, static_cast<int>(n));
    P.alpha_given = 1;
    const dim3 grid(P.nb), blk(kBlock);
    // set up the inputs every kernel reads: slots / block stats (k_correspond), alpha (k_pko), partials; kernel 4 (the
    // correspondence launch with NO setup pass: its inputs not pre-read into the caches) skips it
    if (kernel_id == 5) {                                // the launches' own span (P.span), not the events'
        rc = reset_spans(c);
        if (rc != LO_OK) return rc;
        P.span = c->d_span + static_cast<size_t>(kSpanWords) * kStageEvents;
    }
    if (kernel_id < 4) {
        launch_correspond(c, P, 1, c->kd);
        hipLaunchKernelGGL(k_accumulate, dim3(P.nb_acc), blk, 0, c->stream, P, 0, 0);
    }
    LO_HIP(c, hipGetLastError());
    LO_HIP(c, hipEventRecord(c->ev0, c->stream));
    for (int r = 0; r < reps; ++r) {
        switch (kernel_id) {
            case 0: case 4: case 5: launch_correspond(c, P, 0, c->kd); break;   // KDTree: kNN + fallback + plane fit
            case 1: hipLaunchKernelGGL(k_accumulate, dim3(P.nb_acc), blk, 0, c->stream, P, 0,
                                       P.nb_acc <= kFuseMaxBlocks ? 2 : 0); break;
            case 2: if (spec_ok(P)) launch_pko_spec(c, P, 1); else launch_pko(c, P, 1); break;
            default: hipLaunchKernelGGL(k_solve, dim3(1), dim3(kSolveThreads), 0, c->stream, P, 0, 1); break;
        }
    }
    LO_HIP(c, hipEventRecord(c->ev1, c->stream));
    LO_HIP(c, hipGetLastError());
    LO_HIP(c, hipEventSynchronize(c->ev1));
    float ms = 0.0f;
    LO_HIP(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    *avg_ms = ms / reps;
    if (kernel_id == 5) {
        std::vector<unsigned long long> h(kSpanWords);
        LO_HIP(c, hipMemcpy(h.data(), c->d_span + static_cast<size_t>(kSpanWords) * kStageEvents,
                            kSpanWords * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        const unsigned long long d = span_of(h.data());
        *avg_ms = d ? static_cast<float>(static_cast<double>(d) * 1e-5) : -1.0f;   // the last launch's span
    }
    return LO_OK;
}

int lo_bench_correspond_rr(lo_ctx* const* ctxs, const float* const* d_pts, const size_t* n, const float* T, int count,
                           int rounds, float* avg_ms) {
    if (!ctxs || !d_pts || !n || !T || !avg_ms || count < 1 || rounds < 1) return LO_ERR_ARG;
    lo_ctx* c0 = ctxs[0];
    if (!c0) return LO_ERR_ARG;
    std::vector<KParams> P(count);
    for (int i = 0; i < count; ++i) {
        lo_ctx* c = ctxs[i];
        if (!c || !d_pts[i] || n[i] == 0) return LO_ERR_ARG;
        if (c->kd || c->device != c0->device) { c0->err = "lo_bench_correspond_rr: surfel contexts on one device"; return LO_ERR_STATE; }
        if (n[i] > static_cast<size_t>(c->cfg.max_points)) { c0->err = "n exceeds max_points"; return LO_ERR_CAPACITY; }
    }
    LO_HIP(c0, hipSetDevice(c0->device));
    for (int i = 0; i < count; ++i) {                       // every context's state on its own stream, then joined
        lo_ctx* c = ctxs[i];
        int rc = reset_state(c, T + 12 * i, 1.0, 0.1);
        if (rc == LO_OK) rc = ensure_acc_part(c);
        if (rc != LO_OK) { c0->err = c->err; return rc; }
        P[i] = make_params(c, d_pts[i], static_cast<int>(n[i]));
        LO_HIP(c0, hipStreamSynchronize(c->stream));
    }
    const hipStream_t s = c0->stream;
    LO_HIP(c0, hipEventRecord(c0->ev0, s));
    for (int r = 0; r < rounds; ++r)
        for (int i = 0; i < count; ++i) hipLaunchKernelGGL(k_correspond, dim3(P[i].nb), dim3(kBlock), 0, s, P[i], 0);
    LO_HIP(c0, hipEventRecord(c0->ev1, s));
    LO_HIP(c0, hipGetLastError());
    LO_HIP(c0, hipEventSynchronize(c0->ev1));
    float ms = 0.0f;
    LO_HIP(c0, hipEventElapsedTime(&ms, c0->ev0, c0->ev1));
    *avg_ms = ms / (static_cast<float>(rounds) * count);
    return LO_OK;
}

int lo_seq_sum_f64(lo_ctx* c, const double* x, size_t n, int sort, double* out_sum, long long stats[4]) {
    if (!c || !out_sum || (n > 0 && !x) || n > static_cast<size_t>(kExactMaxPoints)) return LO_ERR_ARG;
    LO_HIP(c, hipSetDevice(c->device));
    double* d = nullptr;
    LO_HIP(c, hipMalloc(&d, (2 * n + 1) * sizeof(double) + 4 * sizeof(long long)));
    long long* d_st = reinterpret_cast<long long*>(d + 2 * n + 1);
    if (n > 0) LO_HIP(c, hipMemcpy(d, x, n * sizeof(double), hipMemcpyHostToDevice));
    launch_seq_sum_diag(d, static_cast<int>(n), sort ? d + n : nullptr, d + 2 * n, d_st, c->stream);
    hipError_t e = hipStreamSynchronize(c->stream);
    long long st[4] = {0, 0, 0, 0};
    if (e == hipSuccess) e = hipMemcpy(out_sum, d + 2 * n, sizeof(double), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(st, d_st, sizeof(st), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) { c->err = std::string("lo_seq_sum_f64: ") + hipGetErrorString(e); return LO_ERR_HIP; }
    if (stats) for (int k = 0; k < 4; ++k) stats[k] = st[k];
    return LO_OK;
}

int lo_seq_sum_f32(lo_ctx* c, const float* x, size_t n, float* out_sum, long long stats[4]) {
    if (!c || !out_sum || (n > 0 && !x) || n > static_cast<size_t>(kMaxBlocks) * kBlock) return LO_ERR_ARG;
    LO_HIP(c, hipSetDevice(c->device));
    const int ni = static_cast<int>(n);
    const size_t x_bytes = (n * sizeof(float) + 255) / 256 * 256, mwb = mw_bytes(1, ni);
    char* d = nullptr;
    LO_HIP(c, hipMalloc(&d, x_bytes + mwb + 256));
    float* d_x = reinterpret_cast<float*>(d);
    const MwBuf B = mw_layout(d + x_bytes, 1, ni);
    float* d_out = reinterpret_cast<float*>(d + x_bytes + mwb);
    long long* d_st = reinterpret_cast<long long*>(d + x_bytes + mwb + 64);
    hipError_t e = hipSuccess;
    if (n > 0) e = hipMemcpy(d_x, x, n * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = mw_clear(B, 1, c->stream);
    float ms = 0.0f;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) {
        (void)hipEventRecord(e0, c->stream);
        launch_mw_sums(d_x, ni, 1, ni, nullptr, nullptr, B, d_out, d_st, c->stream, false);
        (void)hipEventRecord(e1, c->stream);
        e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    long long st[3] = {0, 0, 0};
    if (e == hipSuccess) e = hipMemcpy(out_sum, d_out, sizeof(float), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(st, d_st, sizeof(st), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) { c->err = std::string("lo_seq_sum_f32: ") + hipGetErrorString(e); return LO_ERR_HIP; }
    if (stats) {
        for (int k = 0; k < 3; ++k) stats[k] = st[k];
        stats[3] = static_cast<long long>(ms * 1e3);      // microseconds of the three launches
    }
    return LO_OK;
}

int lo_debug_counters(lo_ctx* c, unsigned long long out[16]) {
    if (!c || !out) return LO_ERR_ARG;
    LO_HIP(c, sync_all(c));
    const DevState* st = c->d_st;
    LO_HIP(c, hipMemcpy(out, reinterpret_cast<const char*>(st) + offsetof(DevState, dbg), 16 * sizeof(unsigned long long),
                        hipMemcpyDeviceToHost));
    return LO_OK;
}

int lo_debug_counters_ex(lo_ctx* c, unsigned long long* out, int n) {
    if (!c || !out || n < 1 || n > 24) return LO_ERR_ARG;
    LO_HIP(c, sync_all(c));
    LO_HIP(c, hipMemcpy(out, reinterpret_cast<const char*>(c->d_st) + offsetof(DevState, dbg),
                        static_cast<size_t>(n) * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return LO_OK;
}

int lo_pko_sample_indices_host(size_t n, int sample_size, int32_t* out) {
    if (!out || sample_size < 1 || sample_size > kMaxS || n > static_cast<size_t>(kMaxBlocks) * kBlock) return LO_ERR_ARG;
    PkoTables t;
    build_pko_tables(t, sample_size, 1, static_cast<int>(std::max<size_t>(n, 1)), 0.1, 10.0, 1, 10.0, false);
    const int k = static_cast<int>(std::min<size_t>(n, static_cast<size_t>(sample_size)));
    for (int s = 0; s < k; ++s) out[s] = pko_sample_host(t, static_cast<int>(n), s);
    return k;
}

}  // extern "C"

// ---------------------------------------------------------------- scan-parallel batch (one GPU)
// B contexts advance through optimize() in lockstep: one launch per kernel per GN iteration for all jobs
// (blockIdx.y = job).  The per-job KParams live in device memory (the batched kernels read them with scalar
// loads); they are rebuilt on the host every call but uploaded only when a job's scan pointer, size or map
// table changed.  The initial poses travel in a separate 12-float-per-job array (KParams::T0p).
static constexpr int kBatchPkoWGs = 256;    // PKO workgroups per launch over all jobs (>= 1 per job; measured best)
// one single-wave PKO workgroup per job (k_pko_tb<1, true>) is opt-in (LO_BATCH_ONE_WAVE=1): with the JS phase's
// LDS alpha table the four-wave split wins at every measured size (2048 jobs 946k vs 828k scans/s, 4096 1.039M vs
// 1.021M); the one-wave variant stays tested (tests/test_gpu_batch.py) for batches beyond the measured range
static constexpr int kBatchOneWaveMin = 0x7fffffff;
// from this many small jobs the accumulate and the solve are two launches (k_accumulate_b1<false> + k_solve_b1):
// the fused form's fp64 solve holds the 8-wave accumulate at 128 VGPRs (2 workgroups per CU; split: 70, 3 per CU).
// Measured: 4096 jobs 1.037M -> 1.090M scans/s, 1024 857k -> 875k; at 64-256 jobs the extra launch costs ~1 %.
static constexpr int kBatchSplitSolveMin = 1024;

struct lo_batch {
    std::vector<lo_ctx*> ctx;
    int device = 0;
    int max_iters = 0;
    int pko_max = 1;                 // min over contexts of the single-scan PKO grid
    int pko_budget = kBatchPkoWGs;   // PKO workgroups per launch over all jobs (LO_BATCH_PKO_WGS overrides)
    int one_wave_min = kBatchOneWaveMin;   // jobs from which PKO runs one wave per job (LO_BATCH_ONE_WAVE=0/1 forces)
    int split_solve_min = kBatchSplitSolveMin;   // jobs from which k_solve_b1 solves (LO_BATCH_FUSED_SOLVE=0/1 forces)
    hipStream_t stream = nullptr;
    std::string err;
    KParams* d_P = nullptr;
    KParams* h_P = nullptr;          // pinned staging of the active jobs' params
    float* d_T0 = nullptr;
    float* h_T0 = nullptr;           // pinned
    lo_batch_rec* d_rec = nullptr;
    lo_batch_rec* h_rec = nullptr;   // pinned
    std::vector<float> T_in;         // count x 12 (T_out of failed / skipped jobs)
    std::vector<int> act;            // active job -> job index
    std::vector<size_t> n;
    struct Sig {
        const lo_ctx* ctx; uint64_t gen; const float* pts; int n; const Slot* tab; uint32_t log2cap; int exact;
        // field by field: the padding after n is not initialised, so a byte compare could report a change every call
        bool operator==(const Sig& o) const {
            return ctx == o.ctx && gen == o.gen && pts == o.pts && n == o.n && tab == o.tab && log2cap == o.log2cap &&
                   exact == o.exact;
        }
    };
    std::vector<Sig> sig;            // what d_P currently holds, per active slot
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev_go = nullptr;      // reference-exact jobs: the batch's uploads done (their streams wait on it)
    std::vector<hipEvent_t> ev_ex;   //   and each exact job's scan finished (the batch stream waits on them)
    int nlock = 0;                   // jobs of the last call that ran in lockstep (the first nlock params)
    bool pending = false;
};

#define LO_BHIP(b, call)                                                                   \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) {                                                            \
            (b)->err = std::string(#call) + ": " + hipGetErrorString(e_);                 \
            return LO_ERR_HIP;                                                             \
        }                                                                                  \
    } while (0)

static int batch_alloc(lo_batch* b) {
    const size_t B = b->ctx.size();
    LO_BHIP(b, hipSetDevice(b->device));
    LO_BHIP(b, hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
    LO_BHIP(b, hipMalloc(&b->d_P, B * sizeof(KParams)));
    LO_BHIP(b, hipHostMalloc(&b->h_P, B * sizeof(KParams), hipHostMallocDefault));
    LO_BHIP(b, hipMalloc(&b->d_T0, B * 12 * sizeof(float)));
    LO_BHIP(b, hipHostMalloc(&b->h_T0, B * 12 * sizeof(float), hipHostMallocDefault));
    LO_BHIP(b, hipMalloc(&b->d_rec, B * sizeof(lo_batch_rec)));
    LO_BHIP(b, hipHostMalloc(&b->h_rec, B * sizeof(lo_batch_rec), hipHostMallocDefault));
    LO_BHIP(b, hipEventCreate(&b->ev0));
    LO_BHIP(b, hipEventCreate(&b->ev1));
    LO_BHIP(b, hipEventCreateWithFlags(&b->ev_go, hipEventDisableTiming));
    LO_BHIP(b, hipFuncSetAttribute(reinterpret_cast<const void*>(k_pko_tb<4, false>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kMaxBlocks * sizeof(int))));
    LO_BHIP(b, hipFuncSetAttribute(reinterpret_cast<const void*>(k_pko_tb<1, true>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kMaxBlocks * sizeof(int))));
    LO_BHIP(b, hipFuncSetAttribute(reinterpret_cast<const void*>(k_exact_acc_b), hipFuncAttributeMaxDynamicSharedMemorySize,
                                   static_cast<int>(kXcLdsBytes)));
    // reference-exact jobs' iteration-0 scale (k_exact_scale_cb, up to 80 KB of dynamic LDS): a process that only
    // batches must not depend on a single-context exact optimize having set the attribute first
    LO_BHIP(b, exact_scale_c_prepare());
    b->T_in.assign(B * 12, 0.0f);
    b->n.assign(B, 0);
    return LO_OK;
}

extern "C" {

lo_batch* lo_batch_create(lo_ctx* const* ctxs, int count, int* err) {
    auto fail = [&](int rc, const char* msg) -> lo_batch* {
        std::fprintf(stderr, "lo_batch_create: %s\n", msg);
        if (err) *err = rc;
        return nullptr;
    };
    if (!ctxs || count < 1 || count > 65535) return fail(LO_ERR_ARG, "need 1..65535 contexts");
    for (int j = 0; j < count; ++j) {
        const lo_ctx* c = ctxs[j];
        if (!c) return fail(LO_ERR_ARG, "null context");
        if (c->kd) return fail(LO_ERR_ARG, "batched optimize needs surfel-mode contexts");
        if (c->device != ctxs[0]->device) return fail(LO_ERR_ARG, "contexts on different devices");
        if (c->cfg.max_iterations != ctxs[0]->cfg.max_iterations) return fail(LO_ERR_ARG, "max_iterations differ");
        for (int k = 0; k < j; ++k) if (ctxs[k] == c) return fail(LO_ERR_ARG, "a context appears twice");
    }
    lo_batch* b = new lo_batch();
    b->ctx.assign(ctxs, ctxs + count);
    b->device = ctxs[0]->device;
    b->max_iters = ctxs[0]->cfg.max_iterations;
    b->pko_max = kPkoMaxWGs;
    for (const lo_ctx* c : b->ctx) b->pko_max = std::min(b->pko_max, pko_grid(c->cfg));
    if (const char* e = std::getenv("LO_BATCH_PKO_WGS")) b->pko_budget = std::max(1, std::atoi(e));
    if (const char* e = std::getenv("LO_BATCH_ONE_WAVE")) b->one_wave_min = std::atoi(e) ? 1 : 0x7fffffff;
    if (const char* e = std::getenv("LO_BATCH_FUSED_SOLVE")) b->split_solve_min = std::atoi(e) ? 0x7fffffff : 1;
    const int rc = batch_alloc(b);
    if (rc != LO_OK) {
        std::fprintf(stderr, "lo_batch_create: %s\n", b->err.c_str());
        lo_batch_destroy(b);
        if (err) *err = rc;
        return nullptr;
    }
    if (err) *err = LO_OK;
    return b;
}

void lo_batch_destroy(lo_batch* b) {
    if (!b) return;
    (void)hipSetDevice(b->device);
    if (b->stream) (void)hipStreamSynchronize(b->stream);
    for (void* p : {static_cast<void*>(b->d_P), static_cast<void*>(b->d_T0), static_cast<void*>(b->d_rec)})
        if (p) (void)hipFree(p);
    for (void* p : {static_cast<void*>(b->h_P), static_cast<void*>(b->h_T0), static_cast<void*>(b->h_rec)})
        if (p) (void)hipHostFree(p);
    if (b->ev0) (void)hipEventDestroy(b->ev0);
    if (b->ev1) (void)hipEventDestroy(b->ev1);
    if (b->ev_go) (void)hipEventDestroy(b->ev_go);
    for (hipEvent_t e : b->ev_ex) (void)hipEventDestroy(e);
    if (b->stream) (void)hipStreamDestroy(b->stream);
    delete b;
}

const char* lo_batch_last_error(const lo_batch* b) { return b ? b->err.c_str() : "null batch"; }
int lo_batch_size(const lo_batch* b) { return b ? static_cast<int>(b->ctx.size()) : 0; }

int lo_batch_optimize_async(lo_batch* b, const float* const* d_pts, const size_t* n, const float* T_init) {
    if (!b || !n || !T_init) return LO_ERR_ARG;
    if (b->pending) { b->err = "batch in flight: call lo_batch_result first"; return LO_ERR_STATE; }
    const int B = static_cast<int>(b->ctx.size());
    for (int j = 0; j < B; ++j) {
        if (n[j] > static_cast<size_t>(b->ctx[j]->cfg.max_points)) { b->err = "n exceeds max_points"; return LO_ERR_CAPACITY; }
        if (b->ctx[j]->cfg.max_iterations != b->max_iters) {   // lo_update_config after lo_batch_create
            b->err = "a context's max_iterations no longer matches the batch's";
            return LO_ERR_STATE;
        }
    }
    LO_BHIP(b, hipSetDevice(b->device));
    for (int j = 0; j < B; ++j) {                      // PKO / candidate buffers first (their pointers go into the params)
        if (n[j] == 0) continue;
        const int rc = ensure_acc_part(b->ctx[j]);
        if (rc != LO_OK) { b->err = b->ctx[j]->err; return rc; }
    }
    std::memcpy(b->T_in.data(), T_init, sizeof(float) * 12 * B);
    b->act.clear();
    int max_nb = 1, max_acc = 1, n_max_ex = 1;
    bool same = true;
    // job order in the device params: the fast-mode jobs, then the reference-exact ones (both in lockstep), then the
    // exact jobs too large for the one-workgroup scale (kExactMergeMax): those run their context's own exact GN loop
    std::vector<int> fast, exl, ex;
    for (int j = 0; j < B; ++j) {
        b->n[j] = n[j];
        if (n[j] == 0) continue;
        lo_ctx* c = b->ctx[j];
        if (!c->exact) fast.push_back(j);
        else if (n[j] <= static_cast<size_t>(kExactMergeMax)) exl.push_back(j);
        else ex.push_back(j);
    }
    const int nfast = static_cast<int>(fast.size()), nexl = static_cast<int>(exl.size());
    for (int pass = 0; pass < 2; ++pass) {
        for (int j : pass ? exl : fast) {
            lo_ctx* c = b->ctx[j];
            const float* pts = (d_pts && d_pts[j]) ? d_pts[j] : c->d_pts;
            const int a = static_cast<int>(b->act.size());
            KParams P = make_params(c, pts, static_cast<int>(n[j]));
            P.T0p = b->d_T0 + 12 * a;
            if (pass) {                                       // the scale comes from k_exact_scale_cb (iteration 0)
                P.scale_given = 1;
                n_max_ex = std::max(n_max_ex, P.n);
            } else {
                max_acc = std::max(max_acc, P.nb_acc);
            }
            max_nb = std::max(max_nb, P.nb);
            const lo_batch::Sig sg{c, c->cfg_gen, pts, P.n, P.tab, P.log2cap, pass};
            if (a >= static_cast<int>(b->sig.size()) || !(b->sig[a] == sg)) same = false;
            if (!same) {
                if (a < static_cast<int>(b->sig.size())) b->sig[a] = sg; else b->sig.push_back(sg);
            }
            b->h_P[a] = P;
            std::memcpy(b->h_T0 + 12 * a, T_init + 12 * j, sizeof(float) * 12);
            b->act.push_back(j);
        }
    }
    const int nact = static_cast<int>(b->act.size());
    b->nlock = nact;
    // large exact jobs after the lockstep ones: only their DevState pointer is read (k_export_batch)
    for (int j : ex) {
        b->h_P[b->act.size()] = make_params(b->ctx[j], b->ctx[j]->d_pts, static_cast<int>(n[j]));
        b->act.push_back(j);
    }
    const int ntot = static_cast<int>(b->act.size());
    if (!ex.empty()) same = false;
    if (static_cast<int>(b->sig.size()) != ntot) { same = false; b->sig.resize(ntot); }
    LO_BHIP(b, hipEventRecord(b->ev0, b->stream));
    if (ntot > 0) {
        if (nact > 0) LO_BHIP(b, hipMemcpyAsync(b->d_T0, b->h_T0, sizeof(float) * 12 * nact, hipMemcpyHostToDevice, b->stream));
        if (!same) LO_BHIP(b, hipMemcpyAsync(b->d_P, b->h_P, sizeof(KParams) * ntot, hipMemcpyHostToDevice, b->stream));
    }
    if (!ex.empty()) {
        // large reference-exact jobs run their context's own exact GN loop (the chip-wide sequential-sum
        // reproductions) on the context stream, ordered after the batch's uploads (lo_batch_optimize copies their
        // points on the batch stream) and before its record export; the scan pipeline stays off for them, so every
        // launch is on the context stream and the record is final when it ends
        LO_BHIP(b, hipEventRecord(b->ev_go, b->stream));
        while (b->ev_ex.size() < ex.size()) {
            hipEvent_t e = nullptr;
            LO_BHIP(b, hipEventCreateWithFlags(&e, hipEventDisableTiming));
            b->ev_ex.push_back(e);
        }
        for (size_t q = 0; q < ex.size(); ++q) {
            const int j = ex[q];
            lo_ctx* c = b->ctx[j];
            const float* pts = (d_pts && d_pts[j]) ? d_pts[j] : c->d_pts;
            LO_BHIP(b, hipStreamWaitEvent(c->stream, b->ev_go, 0));
            const bool pipe = c->pipe, sync_call = c->sync_call;
            c->pipe = false;
            c->sync_call = false;
            const int rc = enqueue_optimize(c, pts, n[j], T_init + 12 * j);
            c->pipe = pipe;
            c->sync_call = sync_call;
            c->pending = false;                               // the batch collects the record, not lo_icp_result
            if (rc != LO_OK) { b->err = std::string("exact job: ") + c->err; return rc; }
            LO_BHIP(b, hipEventRecord(b->ev_ex[q], c->stream));
            LO_BHIP(b, hipStreamWaitEvent(b->stream, b->ev_ex[q], 0));
        }
    }
    if (nact > 0) {
        const int pko_wgs = std::max(1, std::min(b->pko_max, b->pko_budget / nact));
        const size_t pre_bytes = static_cast<size_t>(max_nb) * sizeof(int);
        const dim3 blk(kBlock);
        for (int it = 0; it < b->max_iters; ++it) {
            hipLaunchKernelGGL(k_correspond_b, dim3(max_nb, nact), blk, 0, b->stream, b->d_P, it == 0 ? 1 : 0, it == 0 ? 1 : 0);
            if (it == 0 && nexl > 0) {
                launch_exact_scale_cb(b->d_P + nfast, nexl, n_max_ex, b->stream);
                LO_BHIP(b, hipGetLastError());                 // e.g. a dynamic-LDS launch the attribute did not allow
            }
            if (nact >= b->one_wave_min)
                hipLaunchKernelGGL((k_pko_tb<1, true>), dim3(1, nact), dim3(64), pre_bytes, b->stream, b->d_P, it);
            else
                hipLaunchKernelGGL((k_pko_tb<4, false>), dim3(pko_wgs, nact), dim3(256), pre_bytes, b->stream, b->d_P, it);
            if (nexl > 0)
                hipLaunchKernelGGL(k_exact_acc_b, dim3(nexl), dim3(256), kXcLdsBytes, b->stream, b->d_P + nfast, it);
            if (nfast == 0) continue;
            if (max_acc <= kFuseMaxBlocks) {           // small jobs: one 8-wave workgroup accumulates + solves
                if (nfast < b->split_solve_min) {
                    hipLaunchKernelGGL(k_accumulate_b1<true>, dim3(1, nfast), dim3(512), 0, b->stream, b->d_P, it);
                } else {
                    hipLaunchKernelGGL(k_accumulate_b1<false>, dim3(1, nfast), dim3(512), 0, b->stream, b->d_P, it);
                    hipLaunchKernelGGL(k_solve_b1, dim3(nfast), dim3(kBlock), 0, b->stream, b->d_P, it);
                }
            } else {
                hipLaunchKernelGGL(k_accumulate_b, dim3(max_acc, nfast), blk, 0, b->stream, b->d_P, it);
                hipLaunchKernelGGL(k_solve_b, dim3(nfast), dim3(kSolveThreads), 0, b->stream, b->d_P, it);
            }
        }
    }
    if (ntot > 0) {
        hipLaunchKernelGGL(k_export_batch, dim3(ntot), dim3(64), 0, b->stream, b->d_P, b->d_rec);
        LO_BHIP(b, hipGetLastError());
        LO_BHIP(b, hipMemcpyAsync(b->h_rec, b->d_rec, sizeof(lo_batch_rec) * ntot, hipMemcpyDeviceToHost, b->stream));
    }
    LO_BHIP(b, hipEventRecord(b->ev1, b->stream));
    b->pending = true;
    return LO_OK;
}

int lo_batch_result(lo_batch* b, lo_batch_rec* out, double* gpu_ms) {
    if (!b || !out) return LO_ERR_ARG;
    if (!b->pending) { b->err = "no batch in flight"; return LO_ERR_STATE; }
    LO_BHIP(b, hipSetDevice(b->device));
    LO_BHIP(b, hipStreamSynchronize(b->stream));
    b->pending = false;
    const int B = static_cast<int>(b->ctx.size());
    for (int j = 0; j < B; ++j) {          // skipped jobs: the reference's false on an empty cloud (:593-603)
        lo_batch_rec& R = out[j];
        std::memset(&R, 0, sizeof(R));
        R.status = LO_INSUFFICIENT;
    }
    for (size_t a = 0; a < b->act.size(); ++a) out[b->act[a]] = b->h_rec[a];
    for (int j = 0; j < B; ++j)            // optimized_transform = initial unless the GN loop succeeded (:266, :301)
        if (out[j].status != LO_OK) std::memcpy(out[j].pose, b->T_in.data() + 12 * j, sizeof(float) * 12);
    if (gpu_ms) {
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, b->ev0, b->ev1) != hipSuccess) ms = -1.0f;
        *gpu_ms = ms;
    }
    return LO_OK;
}

int lo_batch_bench_correspond(lo_batch* b, int reps, float* avg_ms) {
    if (!b || reps < 1 || !avg_ms) return LO_ERR_ARG;
    if (b->pending) { b->err = "batch in flight: call lo_batch_result first"; return LO_ERR_STATE; }
    const int nact = b->nlock;
    if (nact == 0) { b->err = "no lockstep batch has run yet"; return LO_ERR_STATE; }
    LO_BHIP(b, hipSetDevice(b->device));
    int max_nb = 1;
    for (int a = 0; a < nact; ++a) max_nb = std::max(max_nb, b->h_P[a].nb);
    const dim3 grid(max_nb, nact), blk(kBlock);
    // every job back at its initial pose with a fresh GN state (init launch), then reps plain launches
    hipLaunchKernelGGL(k_correspond_b, grid, blk, 0, b->stream, b->d_P, 1, 1);
    LO_BHIP(b, hipEventRecord(b->ev0, b->stream));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_correspond_b, grid, blk, 0, b->stream, b->d_P, 0, 0);
    LO_BHIP(b, hipEventRecord(b->ev1, b->stream));
    LO_BHIP(b, hipGetLastError());
    LO_BHIP(b, hipEventSynchronize(b->ev1));
    float ms = 0.0f;
    LO_BHIP(b, hipEventElapsedTime(&ms, b->ev0, b->ev1));
    *avg_ms = ms / reps;
    return LO_OK;
}

int lo_batch_optimize(lo_batch* b, const float* const* pts, const size_t* n, const float* T_init, lo_batch_rec* out) {
    if (!b || !pts || !n || !T_init || !out) return LO_ERR_ARG;
    if (b->pending) { b->err = "batch in flight: call lo_batch_result first"; return LO_ERR_STATE; }
    const int B = static_cast<int>(b->ctx.size());
    LO_BHIP(b, hipSetDevice(b->device));
    for (int j = 0; j < B; ++j) {
        if (n[j] == 0) continue;
        if (!pts[j]) return LO_ERR_ARG;
        if (n[j] > static_cast<size_t>(b->ctx[j]->cfg.max_points)) { b->err = "n exceeds max_points"; return LO_ERR_CAPACITY; }
        LO_BHIP(b, hipMemcpyAsync(b->ctx[j]->d_pts, pts[j], n[j] * 3 * sizeof(float), hipMemcpyHostToDevice, b->stream));
    }
    const int rc = lo_batch_optimize_async(b, nullptr, n, T_init);
    if (rc != LO_OK) return rc;
    return lo_batch_result(b, out, nullptr);
}

}  // extern "C"
