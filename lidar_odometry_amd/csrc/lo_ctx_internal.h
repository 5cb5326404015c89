// lo_ctx_internal.h — library-internal accessors of an ICP context (C++ linkage, not part of the C ABI).
#pragma once
#include <cstdint>

#include "../../include/lo_icp.h"

namespace lo {
// Which host voxel map the context's device surfel table mirrors, and at which journal position / epoch
// (lo_map_sync_voxelmap); src = 0 after any other table upload.
void ctx_map_source(const lo_ctx* c, uint64_t* src, uint64_t* epoch, uint64_t* pos);
void ctx_set_map_source(lo_ctx* c, uint64_t src, uint64_t epoch, uint64_t pos);

// Device surfel fits for a host map's deferred jobs (lo_voxelmap_set_device_fit).  ctx_fit_surfels fits job j over
// cs[3 * offs[j] ...) (children up to offs[j + 1], the last to n_cs) with k_surfel_fit on the context stream, which
// patches the table (upsert when planarity <= thr, else erase) after any patch already enqueued, and copies the
// results back asynchronously; *ticket identifies the launch.  LO_ERR_CAPACITY if the table could overflow (the
// caller then fits on the host and uploads everything).  ctx_fit_results waits for that launch and returns its
// results; LO_ERR_STATE if the context is gone or has launched other fits since (the caller fits on the host).
struct FitResult {
    float n[3];
    float c[3];
    float planarity;
    uint32_t pad;
};
int ctx_fit_surfels(lo_ctx* c, const int32_t* keys, const int32_t* offs, size_t n_jobs, const float* cs, size_t n_cs,
                    float thr, uint64_t* ticket);
int ctx_fit_results(lo_ctx* c, uint64_t ticket, FitResult* out, size_t n_jobs);

// Device map (lo_devmap): the context's surfel table with at least min_slots slots, emptied (asynchronously, on the
// context stream) unless it is still the generation the map reserved last time; *gen changes whenever the table was
// emptied, so the map refills it.  Any other upload to the context bumps the generation.
int ctx_reserve_table(lo_ctx* c, size_t min_slots, void** tab, uint32_t* log2cap, uint64_t* gen);
// The device-filtered scan of the last lo_icp_optimize_raw / lo_voxel_filter_gpu: device points and the device
// count (stream-ordered; no sync).
int ctx_filtered_device(lo_ctx* c, const float** d_pts, const int** d_n);
// KDTree contexts (use_surfel_correspondence = 0): the correspondence grid (lo_map_set_points' RebuildKdTree
// equivalent) built on the device from a device point array -- the device map's L0 centroids in GetPointCloud order:
// xyz (3 floats per point), *d_count of them (<= cap).  One small readback (count and bounds) sizes the grid; the
// cell sort is a stable device radix sort, so the grid equals lo_map_set_points' on the same points.  No kd visit
// order is built: a query that meets a deciding distance tie flags it, and lo_icp_result rebuilds the grid with the
// order on the host and re-runs that scan (rare: equal distances between distinct centroids).
int ctx_grid_from_device(lo_ctx* c, const float* d_xyz, const int* d_count, size_t cap);
}  // namespace lo
