/*
 * lo_icp.h — C ABI of the MI355X-native point-to-plane ICP registration core.
 *
 * Drop-in boundary for the reference's scan-to-map Gauss-Newton step:
 *   bool IterativeClosestPointOptimizer::optimize(map::VoxelMap*, shared_ptr<LidarFrame>,
 *                                                 const SE3f& initial, SE3f& optimized)
 *   (reference src/optimization/IterativeClosestPointOptimizer.h:182-185, .cpp:255-463)
 * and the map queries it makes:
 *   VoxelMap::GetSurfelAtPoint       (src/database/VoxelMap.h:252-254, VoxelMap.cpp:368-386)
 *   AdaptiveMEstimator::calculate_scale_factor (src/optimization/AdaptiveMEstimator.h:92, .cpp:63-79)
 *
 * Conventions (no exceptions cross this boundary; plain pointers and sizes only):
 *  - A context = one GPU + one HIP stream + device-resident map, scan buffers and PKO tables.
 *    Contexts are not thread-safe; distinct contexts may run concurrently (scan-parallel multi-GPU).
 *  - The caller owns every host buffer; the library owns every device buffer.
 *  - Poses are fp32 row-major 3x4 [R|t] (SE3f::Matrix() rows 0-2).
 *  - Points are AoS float3 (util::Point3D, PointCloudUtils.h:34-38), local (sensor) frame.
 *  - Return codes: LO_OK (0); LO_INSUFFICIENT (1) = a GN iteration found fewer than
 *    min_correspondence_points correspondences (the reference's `return false`, T_out = T_init);
 *    negative = argument / HIP errors (lo_last_error() has the text).
 */
#ifndef LO_ICP_H
#define LO_ICP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LO_OK              0
#define LO_INSUFFICIENT    1
#define LO_ERR_ARG        -1
#define LO_ERR_HIP        -2
#define LO_ERR_CAPACITY   -3
#define LO_ERR_STATE      -4
#define LO_ERR_PIPELINE   -5   /* device-side status only: a scan-pipeline wait timed out (lo_pipeline_status) */

#define LO_MAX_ITERS      64

/* PKO kernel types (AdaptiveMEstimatorConfig::pko_kernel_type, AdaptiveMEstimator.h:40; the weights of
 * pko_kernel_weight, AdaptiveMEstimator.cpp:99-156).  Any other name selects Cauchy there, as lo_pko_kernel_from_name. */
#define LO_PKO_HUBER          0
#define LO_PKO_CAUCHY         1
#define LO_PKO_TUKEY          2
#define LO_PKO_WELSCH         3
#define LO_PKO_GEMAN_MCCLURE  4
#define LO_PKO_PSEUDO_HUBER   5

/* ICPConfig (IterativeClosestPointOptimizer.h:55-76, wired by Estimator.cpp:62-70) +
 * AdaptiveMEstimatorConfig (AdaptiveMEstimator.h:24-41, built at Estimator.cpp:49-59) +
 * the map geometry the surfel lookup needs (VoxelMap::GetVoxelSize/GetHierarchyFactor, VoxelMap.h:204-205). */
typedef struct lo_config {
    int    max_iterations;               /* config/kitti.yaml:35 -> 4 */
    double translation_tolerance;        /* 0.005 m */
    double rotation_tolerance;           /* 0.005 rad */
    double max_correspondence_distance;  /* 1.0 m */
    int    min_correspondence_points;    /* 10 (ICPConfig default; estimator.min_correspondence_points is not wired) */
    int    use_robust_loss;              /* 1 */
    double robust_loss_delta;            /* 0.1, used only when PKO is disabled */
    int    loss_cauchy;                  /* 0: huber weight (SystemConfig.loss_type is never parsed -> "huber") */
    int    use_adaptive_m_estimator;     /* 1: PKO */
    double min_scale_factor;             /* 0.1 */
    double max_scale_factor;             /* 10.0 */
    int    num_alpha_segments;           /* 100 */
    double truncated_threshold;          /* 10.0 */
    int    gmm_components;               /* 3 (1..3 supported) */
    int    gmm_sample_size;              /* 100 (1..256 supported) */
    int    pko_kernel;                   /* LO_PKO_*: pko_kernel_type, "huber" in kitti.yaml:51 / mid360.yaml:51 */
    float  voxel_size;                   /* map_voxel_size 0.5 */
    int    hierarchy_factor;             /* 3 */
    int    use_surfel_correspondence;    /* 1: L1 surfel lookup; 0: KDTree variant (5-NN plane fit, :647-767) */
    int    max_points;                   /* scan capacity (points per optimize call) */
} lo_config;

/* One executed Gauss-Newton iteration (per-iteration parity log). */
typedef struct lo_iter_log {
    float  pose[12];   /* pose after this iteration's update */
    int    n_corr;
    double scale;      /* iteration-0 residual normalisation scale (std/6) */
    double alpha;      /* PKO Huber delta used for the weights */
    float  cost;       /* sum w r^2 */
    float  H[21];      /* upper triangle of H, row-major */
    float  g[6];
    float  delta[6];   /* [dt, dw] */
} lo_iter_log;

typedef struct lo_stats {
    int    iterations;
    int    n_corr;         /* last iteration */
    int    status;         /* LO_OK / LO_INSUFFICIENT */
    int    converged;      /* reference always reports true (IterativeClosestPointOptimizer.cpp:456) */
    double initial_cost;
    double final_cost;
    double gpu_ms;         /* device time of the whole optimize (HIP events) */
} lo_stats;

typedef struct lo_ctx lo_ctx;

void        lo_config_default_kitti(lo_config* cfg);
/* pko_kernel_type string -> LO_PKO_* exactly as pko_kernel_weight dispatches (AdaptiveMEstimator.cpp:128-156):
 * "huber", "cauchy", "tukey", "welsch", "gemanMcClure", "pseudoHuber"; anything else (NULL included) -> Cauchy. */
int         lo_pko_kernel_from_name(const char* name);
void        lo_config_default_mid360(lo_config* cfg);
lo_ctx*     lo_create(const lo_config* cfg, int device, int* err);
void        lo_destroy(lo_ctx* ctx);
const char* lo_last_error(const lo_ctx* ctx);
int         lo_device(const lo_ctx* ctx);
int         lo_get_config(const lo_ctx* ctx, lo_config* out);   /* the configuration the context was built with */

/* ---- map side ----
 * Replaces the map state read by VoxelMap::GetSurfelAtPoint: the L1 voxels with has_surfel == true.
 * keys_xyz: int32 L1 voxel keys (VoxelKey, VoxelMap.h:152-164), |key| < 2^20 per axis.
 * Full upload; call again after every VoxelMap::UpdateVoxelMap (Estimator.cpp:457). */
int lo_map_set_surfels(lo_ctx* ctx, const int32_t* keys_xyz, const float* normals, const float* centroids, size_t m);
/* Incremental form: the L1 voxels an UpdateVoxelMap changed, patched into the device table in place
 * -- present[i] = 1: voxel i has a surfel (inserted, or its normal / centroid refitted), 0: it lost it or was erased
 * (VoxelMap.cpp:187-261).  Asynchronous on the context stream, no full-table rebuild or host sync.  Returns
 * LO_ERR_CAPACITY (nothing changed) when the table's load, tombstones included, would pass 1/2: upload the whole
 * map with lo_map_set_surfels instead. */
int lo_map_patch_surfels(lo_ctx* ctx, const int32_t* keys_xyz, const float* normals, const float* centroids,
                         const uint8_t* present, size_t m);
/* The reference-side sync after UpdateVoxelMap (Estimator.cpp:457) for a caller that keeps the reference's own VoxelMap:
 * the map's whole current surfel set (GetL1Surfels, VoxelMap.cpp:405-418, filed under L1 keys) is diffed on the host
 * against the set this context last received through this call, and only the difference -- new or refitted surfels,
 * surfels that left (VoxelMap.cpp:187-261) -- is patched into the device table in place (lo_map_patch_surfels), so
 * the device work is O(changed voxels).  The first call, a table changed by anything else since, or a table too full
 * for the patch upload everything (lo_map_set_surfels).  patched (nullable): records sent, -1 after a full upload. */
int lo_map_sync_surfels(lo_ctx* ctx, const int32_t* keys_xyz, const float* normals, const float* centroids, size_t m,
                        int* patched);
size_t lo_map_surfel_count(const lo_ctx* ctx);

/* KDTree variant (use_surfel_correspondence = 0): the map point cloud the reference's kd-tree indexes,
 * VoxelMap::GetPointCloud (VoxelMap.cpp:388-403) = L0 centroids in L0 order.  Replaces
 * VoxelMap::RebuildKdTree (:420-438, called at Estimator.cpp:461) with a device grid built from it.
 * Neighbour ties are broken by this order (index).  LO_ERR_STATE on a surfel-mode context. */
int lo_map_set_points(lo_ctx* ctx, const float* xyz, size_t m);
/* Scans re-run because a device-built KDTree grid (the device map's, lo_devmap_sync_points) met a deciding distance
 * tie: lo_icp_result then builds the kd visit order on the host and optimizes the scan again. */
int lo_kd_reruns(const lo_ctx* ctx);
size_t lo_map_point_count(const lo_ctx* ctx);

/* ---- the optimize boundary ----
 * Same contract as IterativeClosestPointOptimizer::optimize: GN to convergence / max_iterations.
 * logs: nullable, room for cfg.max_iterations entries; stats: nullable. Synchronous. */
int lo_icp_optimize(lo_ctx* ctx, const float* pts_xyz, size_t n, const float T_init[12], float T_out[12],
                    lo_iter_log* logs, lo_stats* stats);

/* Device-resident variant: d_pts is a device pointer (AoS float3) on the context's device.
 * Enqueues the whole GN loop on the context stream and returns immediately; the result is
 * read (and the stream synchronised) by lo_icp_result(). */
int lo_icp_optimize_async(lo_ctx* ctx, const float* d_pts, size_t n, const float T_init[12]);
int lo_icp_result(lo_ctx* ctx, float T_out[12], lo_iter_log* logs, lo_stats* stats);
/* stats->gpu_ms: the device time of a synchronous call (HIP events around its launches); -1 after an async call,
 * which records no events (each marker packet costs several us of device time between two kernels). */
int lo_sync(lo_ctx* ctx);
void* lo_stream(lo_ctx* ctx);   /* hipStream_t of the context */
/* Run the context on a caller stream (e.g. the framework's current stream); NULL = own stream again (a fresh
 * hipStreamNonBlocking stream -- so the legacy default stream, handle 0, cannot be selected: pass a created stream). */
int lo_set_stream(lo_ctx* ctx, void* hip_stream);
/* Arithmetic mode.  enable = 1 (THE DEFAULT of every context): reference-exact -- H, g and the cost summed
 * SEQUENTIALLY in fp32 over the correspondences in scan order, the iteration-0 scale from the sorted residuals, the
 * fp32 LDLT and SO3 re-projection through JacobiSVD: the reference's own operation order
 * (IterativeClosestPointOptimizer.cpp:304-449, MathUtils.cpp:23-99), so the per-iteration logs equal the oracle
 * restatement's bit for bit (the sequential sums are reproduced in parallel, lo_seqsum.h).  enable = 0: the fast mode
 * (opt-in) -- fixed-order fp64 tree sums, a Chan-merged scale, an fp64 LDLT with a polar SO3 projection; within 1e-7
 * of the reference per step, but a PKO alpha near-tie or a correspondence on a voxel face can then resolve the other way
 * and move the pose by 1e-4 .. 4e-4 (measured on the MID360-like and 1M-point workloads): NOT parity-safe.
 * LO_EXACT=0 in the environment starts contexts in the fast mode (A/B runs).
 * Device memory of the exact mode, allocated at the first scan that needs it and kept: up to 16384 points a fixed
 * ~3 MB; a larger scan adds ~0.85 KB per point of the largest such scan (the 14 fp32 factor rows the 43 terms are
 * formed from, 56 B, and the sequential-sum head records, 2 x 1024 per 4096-term chunk of every column at 36 B,
 * ~775 B) -- ~0.85 GB at 1M points, ~3.4 GB at the 4M-point max_points.  An allocation failure there returns LO_ERR_HIP from that optimize call. */
int lo_set_exact(lo_ctx* ctx, int enable);
/* Scan pipeline (default on; LO_PIPE=0 in the environment turns it off at lo_create).  The reference's optimize
 * runs GN iterations until convergence (IterativeClosestPointOptimizer.cpp:281-449); the device loop enqueues all
 * max_iterations and a converged scan's later launches leave early.  With the pipeline, iterations >= main_iterations
 * (default 2) of a small surfel scan with PKO go to a second stream of the context, and the context stream waits on
 * the device only until the scan's result is final: the early-exit launches of a converged scan drain beside the
 * next scan instead of in front of it.  Results are identical with the pipeline on or off; everything enqueued on
 * the context stream after an optimize sees its final result; lo_sync drains both streams.  main_iterations 0 keeps
 * the current split. */
int lo_set_pipeline(lo_ctx* ctx, int enable, int main_iterations);
/* IterativeClosestPointOptimizer::update_config (IterativeClosestPointOptimizer.h:220): new parameters, same context --
 * the device map, buffers and stream stay.  voxel_size, hierarchy_factor, max_points and use_surfel_correspondence
 * are fixed at lo_create (LO_ERR_STATE); new PKO parameters rebuild the PKO tables. */
int lo_update_config(lo_ctx* ctx, const lo_config* cfg);
/* Workgroups of a PKO launch that fit the GMM (each fits it redundantly, then evaluates its share of the alpha grid):
 * 0 (default, LO_PKO_GROUPS) = one alpha each (the latency-optimal single-stream shape); fewer leave the chip to other
 * contexts' launches when many sequences share a GPU.  Results are identical for every value. */
int lo_set_pko_groups(lo_ctx* ctx, int groups);
/* Scan-pipeline state: out[0] enabled, out[1] main iterations, out[2] timeouts (a device-side wait gave up -- the two
 * streams were not run concurrently -- and the pipeline was switched off), out[3] synchronous scans re-run on one
 * stream after a timeout.  A scan whose wait timed out reports LO_ERR_PIPELINE in its device status (the exported
 * record of an async scan); lo_icp_result re-runs it on one stream instead of returning that status.  That re-run reads
 * the points of the context's LAST enqueued scan again: after lo_icp_optimize_async / lo_icp_optimize_raw_async the
 * caller's device buffer (d_pts / d_raw, and the device count) must therefore stay valid and unchanged until
 * lo_icp_result has returned -- the same lifetime a stream-ordered reader of the buffer needs anyway.  Earlier async
 * scans are never re-run: their exported records keep LO_ERR_PIPELINE. */
int lo_pipeline_status(lo_ctx* ctx, int out[4]);
/* In-step timing: with enable, each optimize brackets its FIRST correspondence launch (k_correspond, or the KDTree
 * k_knn + k_knn_brute + k_plane) with HIP events on the context stream (up to 1024 scans; enabling resets them).
 * lo_stage_time syncs the stream and returns the average in-step duration (us) and the number of timed scans. */
int lo_set_stage_timing(lo_ctx* ctx, int enable);
int lo_stage_time(lo_ctx* ctx, double* avg_us, int* count);
/* The same timed launches' own execution spans (surfel correspondence: first block's start to last block's end,
 * s_memrealtime at 100 MHz inside k_correspond) -- what a kernel trace reports, without the dispatch latency the HIP
 * events add (several us, a large share of a ~13 us 1M-point launch).  Syncs the stream. */
int lo_stage_span(lo_ctx* ctx, double* avg_us, int* count);
/* With stage timing on, the lead PKO workgroup also clocks its EM loop (s_memtime): out = {cycles, EM iterations, fits}
 * summed over the optimize calls since the last reset (the dominant kernel's cycles per EM iteration, measured in the
 * running GN loop).  Syncs the stream; reset != 0 zeroes the sums. */
int lo_pko_em_stats(lo_ctx* ctx, unsigned long long out[3], int reset);
/* Enqueue a copy of the current GN state into device memory: 16 floats = pose[12], status, iterations,
 * n_corr, 0.  For the scan-parallel pose gather (RCCL all-gather of these 16 floats per rank). */
int lo_icp_export_pose(lo_ctx* ctx, float* d_out16);
/* Timing harness: reps back-to-back launches of one kernel (0 correspond, 1 accumulate, 2 pko, 3 solve; 4 correspond
 * without the set-up pass the others get, so a scan last touched long ago is read from HBM) on a device-resident scan
 * at pose T; writes the average device time per launch (HIP events).  5: as 4, timed by the last launch's own span
 * (lo_stage_span's clock: the first blocks' start to the last blocks' end; surfel correspondence only). */
int lo_bench_kernel(lo_ctx* ctx, const float* d_pts, size_t n, const float T[12], double scale, double alpha,
                    int kernel_id, int reps, float* avg_ms);
/* Timing harness for the out-of-cache correspondence roofline: `rounds` round-robin passes over `count` contexts,
 * one correspondence launch per context per pass (d_pts[i], n[i] points at pose T[12 i .. 12 i + 11]), every launch
 * back to back on ctxs[0]'s stream with no set-up pass, so each scan was last touched count - 1 launches earlier.  HIP
 * events around the whole sequence: avg_ms = device time per launch, including the inter-launch gap of back-to-back
 * dispatches (what a kernel trace's per-launch duration plus its dispatch gap adds up to).  Surfel contexts on one
 * device; the caller's streams are not used. */
int lo_bench_correspond_rr(lo_ctx* const* ctxs, const float* const* d_pts, const size_t* n, const float* T, int count,
                           int rounds, float* avg_ms);

/* ---- scan-parallel batch on one GPU ----
 * The north star's scan-parallel model (one independent scan stream per GPU, BASELINE.json configs[4]) applied
 * inside one GPU: B contexts on the same device -- B independent sequences, each with its own map, scan buffer
 * and GN state -- advance through optimize() in lockstep, one launch per kernel per GN iteration for all B
 * (blockIdx.y = job).  Each job computes exactly what lo_icp_optimize computes on its context (bit-identical:
 * same kernels, same per-job reductions).  The reference has no batch entry point; this is the multi-sequence
 * form of IterativeClosestPointOptimizer::optimize (IterativeClosestPointOptimizer.cpp:255-463) called once
 * per sequence.  Requirements: surfel correspondence mode, one device, equal max_iterations.  A context in
 * reference-exact mode (lo_set_exact) runs its own exact GN loop on its context stream inside the batch call (the
 * sequential-sum reproductions have no lockstep form), ordered after the batch's uploads and before its record
 * export, bit-identical to its lo_icp_optimize.  The batch runs on its own stream; the contexts must be idle while
 * it runs and each context's lo_icp_result() is not valid for a batched scan (use lo_batch_result). */
typedef struct lo_batch lo_batch;
typedef struct lo_batch_rec {
    float  pose[12];       /* optimized pose (T_init when status != LO_OK, as lo_icp_optimize) */
    int    status;         /* LO_OK / LO_INSUFFICIENT */
    int    iterations;
    int    n_corr;         /* last iteration */
    float  initial_cost;
    float  final_cost;
    float  pad;
    double alpha;          /* last PKO Huber delta */
} lo_batch_rec;
lo_batch*   lo_batch_create(lo_ctx* const* ctxs, int count, int* err);
void        lo_batch_destroy(lo_batch* b);
const char* lo_batch_last_error(const lo_batch* b);
int         lo_batch_size(const lo_batch* b);
/* d_pts[j]: device pointer (AoS float3) of job j's scan, or NULL = the points last uploaded to context j by
 * lo_batch_optimize; n[j] its point count (0 = the job is skipped and reports LO_INSUFFICIENT); T_init: count x 12
 * row-major poses.  Enqueues every job's whole GN loop and returns. */
int lo_batch_optimize_async(lo_batch* b, const float* const* d_pts, const size_t* n, const float* T_init);
/* Waits for the batch; out[count] receives one record per job.  Returns LO_OK or a negative error. */
int lo_batch_result(lo_batch* b, lo_batch_rec* out, double* gpu_ms);
/* Timing harness: reps back-to-back launches of the batched correspondence kernel over the last batch's jobs at
 * their initial poses (after one resetting launch); writes the average device time per launch (HIP events).
 * Leaves every job's GN state at its initial pose. */
int lo_batch_bench_correspond(lo_batch* b, int reps, float* avg_ms);
/* Host points in, records out (H2D of every scan on the batch stream, enqueue, wait). */
int lo_batch_optimize(lo_batch* b, const float* const* pts, const size_t* n, const float* T_init, lo_batch_rec* out);

/* ---- single-stage entry points (parity harness; each synchronous) ---- */
/* ---- device preprocessing + optimize (Estimator::preprocess_frame, Estimator.cpp:561-588) ----
 * FastVoxelFilter::filter (VoxelMap.h:73-104) on the device -- stride sampling, Morton-cell grouping with the
 * reference's clamp, fp32 sums in point order, output in first-occurrence order, bit-identical -- followed by
 * the optimize loop on the filtered points; the filtered count never leaves the device.
 * ceil(n_raw / stride) must not exceed cfg.max_points. */
int lo_icp_optimize_raw_async(lo_ctx* ctx, const float* d_raw, size_t n_raw, int stride, float voxel_size,
                              const float T_init[12]);
int lo_icp_optimize_raw(lo_ctx* ctx, const float* raw_xyz, size_t n_raw, int stride, float voxel_size,
                        const float T_init[12], float T_out[12], lo_iter_log* logs, lo_stats* stats);
/* Page-locked, device-accessible host memory for raw scans (a sensor driver's ring buffer).  A scan handed to
 * lo_icp_optimize_raw / lo_odom_process in such memory is read by the device filter directly (only the sampled
 * points cross the bus); any other host pointer is staged with one copy of the whole scan. */
void* lo_host_alloc(size_t bytes);
void  lo_host_free(void* p);
/* The last device-filtered scan (the frame's feature cloud, for the keyframe map update); returns the count. */
long long lo_filtered_points(lo_ctx* ctx, float* out_xyz, size_t cap);
/* Filter only (parity): host raw in, host filtered out; returns the count or a negative error. */
long long lo_voxel_filter_gpu(lo_ctx* ctx, const float* raw_xyz, size_t n_raw, float voxel_size, int stride,
                              float* out_xyz, size_t cap);

/* ---- loop-closure ICP (IterativeClosestPointOptimizer::optimize_loop, IterativeClosestPointOptimizer.cpp:40-251;
 * find_correspondences_loop :465-585; called from Estimator.cpp:686, :1001) ----
 * curr / matched: the two keyframes' feature clouds (local frames, AoS float3, host memory) with their world poses.
 * The matched cloud is put in the world (transform_point_cloud) and gridded on the device (a separate grid: the
 * context's own map is untouched, whatever its correspondence mode); then up to 100 GN iterations of exact 5-NN +
 * collinearity gate + plane fit (no distance gate), PKO, normal equations and solve, as optimize_loop.
 * Returns LO_OK when the iteration converged AND the inlier ratio (nearest matched point < 1 m) is >= 0.5 (the
 * reference's true); LO_INSUFFICIENT otherwise (too few correspondences, no convergence in 100 iterations, or
 * too few inliers).  As the reference, T_rel_out = T_curr^-1 * optimized pose and inlier_ratio are written only
 * when the iteration converged (stats->converged = 1).  logs (nullable) receives the first LO_MAX_ITERS
 * iterations. */
int lo_icp_optimize_loop(lo_ctx* ctx, const float* curr_xyz, size_t n_curr, const float T_curr[12],
                         const float* matched_xyz, size_t n_matched, const float T_matched[12],
                         float T_rel_out[12], float* inlier_ratio, lo_iter_log* logs, lo_stats* stats);

/* find_correspondences (IterativeClosestPointOptimizer.cpp:587-645) at pose T:
 * per-point valid flag and fp64 residual |n.(p_w - c)| (0 where invalid). Returns the count. */
int lo_find_correspondences(lo_ctx* ctx, const float* pts_xyz, size_t n, const float T[12],
                            uint8_t* valid, double* residual);
/* KDTree variant's neighbour search (util::KdTree::nearestKSearch(q, 5), PointCloudUtils.h:398-423, over the map
 * cloud set by lo_map_set_points; use_surfel_correspondence = 0): for each world-frame query, the 5 nearest map
 * points by fp32 squared distance, ascending, equal distances in nanoflann's visit order.  idx (n x 5): original
 * map-point indices; dist (n x 5): fp32 squared distances.  A query with fewer than 5 neighbours (the ICP skips it,
 * IterativeClosestPointOptimizer.cpp:699-701) gets idx -1 / dist +inf.  Returns the number of queries with 5. */
int lo_knn_search(lo_ctx* ctx, const float* query_xyz, size_t n, int32_t* idx, float* dist);
/* AdaptiveMEstimator::calculate_scale_factor on given normalised residuals (device PKO).
 * gmm_out (nullable): weights, means, variances (3*gmm_components doubles). Returns alpha, NaN on error. */
double lo_pko_scale_factor(lo_ctx* ctx, const double* residuals, size_t n, double* gmm_out);
/* Weighted normal equations of one GN iteration (IterativeClosestPointOptimizer.cpp:345-410) at pose T
 * with the given normalisation scale and Huber delta. H is 6x6 row-major (fp64 sums). Returns n_corr. */
int lo_build_normal_equations(lo_ctx* ctx, const float* pts_xyz, size_t n, const float T[12],
                              double scale, double delta, double H[36], double g[6], double* cost);
/* PKO sampling: first min(gmm_sample_size, n) entries of std::shuffle(iota(n), mt19937(42))
 * as the device tables reproduce them (AdaptiveMEstimator.cpp:319-328). Host-side. */
int lo_pko_sample_indices(lo_ctx* ctx, size_t n, int32_t* out);
/* Parity entry point of the reference-exact scale (IterativeClosestPointOptimizer.cpp:304-316: std::sort, then
 * std::accumulate): s = 0; s += x[i] in index order (after an ascending sort when sort != 0), one fp64 rounding per
 * addition, for n <= 16384 non-negative doubles -- computed by the device kernel the exact mode uses (lo_seqsum.h).
 * stats (nullable): segment heads (-1: the plain chain ran), fallback segments, fallback terms, device cycles. */
int lo_seq_sum_f64(lo_ctx* ctx, const double* x, size_t n, int sort, double* out_sum, long long stats[4]);
/* Parity entry point of the large-scan exact normal equations (IterativeClosestPointOptimizer.cpp:359-415: running fp32
 * sums in correspondence order): s = 0.0f; s += x[i] in index order, one fp32 rounding per addition, terms of any sign,
 * computed by the device kernels the exact mode uses for scans beyond 16384 points (lo_seqsum.h "Long signed fp32
 * columns": chunk sums, classification, walk).  n <= 4M (the largest scan).  stats (nullable): segment heads, segments
 * summed term by term, chunks run term by term (more heads than a chunk's record list holds), device microseconds. */
int lo_seq_sum_f32(lo_ctx* ctx, const float* x, size_t n, float* out_sum, long long stats[4]);
/* Diagnostic: 16 device counters (phase timestamps of the -DLO_PKO_STAMPS build; zeros otherwise). */
int lo_debug_counters(lo_ctx* ctx, unsigned long long out[16]);
/* Diagnostic: the first n (<= 24) device counters. */
int lo_debug_counters_ex(lo_ctx* ctx, unsigned long long* out, int n);
/* Context-free host variant (no GPU needed): sample_size = gmm_sample_size. */
int lo_pko_sample_indices_host(size_t n, int sample_size, int32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* LO_ICP_H */
