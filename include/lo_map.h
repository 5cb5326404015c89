/*
 * lo_map.h — map-side C ABI: the 2-level voxel/surfel map that feeds the ICP's surfel table, and the
 * scan downsampler that feeds its point cloud.  Host C++ (host form).
 *
 *   lo_voxelmap_*   replaces map::VoxelMap's build side: UpdateVoxelMap (src/database/VoxelMap.cpp:128-262),
 *                   AddPoint (:99-120), surfel PCA + planarity erase (:187-261), GetPointCloud (:388-403).
 *   lo_voxel_filter replaces map::FastVoxelFilter::filter (src/database/VoxelMap.h:73-104).
 *
 * Results are bit-identical to the reference's fp32 arithmetic (insertion-ordered containers with
 * unordered_dense's swap-with-last erase, Eigen JacobiSVD<Matrix3f> restated), checked against the oracle.
 * Every lo_voxelmap_* call (the const readers included: they apply pending device fits) locks the map's recursive
 * mutex, as the reference's VoxelMap does, so one map may be used from several threads.
 */
#ifndef LO_MAP_H
#define LO_MAP_H

#include <stddef.h>
#include <stdint.h>

#include "lo_icp.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lo_voxelmap lo_voxelmap;

lo_voxelmap* lo_voxelmap_create(float voxel_size, int hierarchy_factor, float planarity_threshold, int compute_surfels);
void         lo_voxelmap_destroy(lo_voxelmap* m);
/* UpdateVoxelMap(new_cloud (world frame), sensor_position, max_distance, is_keyframe) */
int          lo_voxelmap_update(lo_voxelmap* m, const float* world_xyz, size_t n, const double sensor[3],
                                double max_distance, int is_keyframe);
/* ApplyTransformAndRehash(T_correction) (VoxelMap.cpp:264-302; called after pose-graph optimisation, Estimator.cpp:877,
 * :1181): every L0 centroid moved by T (row-major 3x4) and re-keyed, collisions merged, surfels recomputed.
 * The next lo_map_sync_voxelmap uploads the whole map. */
int          lo_voxelmap_apply_transform(lo_voxelmap* m, const float T[12]);
/* Device surfel fits: with enable, UpdateVoxelMap records each touched L1 voxel's refit
 * (its children's centroids in child order) instead of fitting on the host; the next lo_map_sync_voxelmap of a
 * context that mirrors this map runs them there (k_surfel_fit: the same fp32 mean / covariance / JacobiSVD code)
 * and patches its table, and the results come back to the map before anything reads it -- surfel fields, or the
 * planarity erase of the voxel and its children in the sequential loop's order.  Bit-identical to enable = 0.
 * Without such a sync the map fits on the host when it is next read. */
int          lo_voxelmap_set_device_fit(lo_voxelmap* m, int enable);
size_t       lo_voxelmap_l0_count(const lo_voxelmap* m);
size_t       lo_voxelmap_l1_count(const lo_voxelmap* m);
size_t       lo_voxelmap_surfel_count(const lo_voxelmap* m);
/* L1 voxels with has_surfel, in L1 iteration order. Returns the number written. */
size_t       lo_voxelmap_get_surfels(const lo_voxelmap* m, int32_t* keys_xyz, float* normals, float* centroids,
                                     float* planarity, size_t cap);
/* The L1 keys whose surfel the last lo_voxelmap_update may have changed -- created, refitted, lost its planarity or
 * its children, erased by the radius prune or the planarity test (VoxelMap.cpp:146-169, :187-261) -- each key once,
 * ordered by key (an update that changed nothing gives none).  What the reference's UpdateVoxelMap
 * collects with the two-line hook INTEGRATION.md shows, for the adapter's keyed sync_map (only these voxels patched:
 * GetSurfelAtPoint at each key's centre, lo_map_patch_surfels).  After lo_voxelmap_apply_transform every key moved:
 * none are listed, upload the whole map.  Returns the count; writes up to cap keys. */
size_t       lo_voxelmap_changed_l1(const lo_voxelmap* m, int32_t* keys_xyz, size_t cap);
/* GetSurfelAtPoint (VoxelMap.cpp:368-386): 1 and the normal / centroid of the surfel of p's L1 voxel
 * (PointToVoxelKey(p, 1)) if it has one, else 0. */
int          lo_voxelmap_surfel_at(const lo_voxelmap* m, const float p[3], float normal[3], float centroid[3]);
/* The keyed sync's lookup loop in one call: for each of n L1 keys, GetSurfelAtPoint at the key's voxel centre
 * ((k + 0.5) * voxel * factor per axis, fp32) -- present[i] = 1 and its normal / centroid, or 0 and zeros.  The
 * arrays go straight to lo_map_patch_surfels.  Returns the number present. */
size_t       lo_voxelmap_surfels_at_keys(const lo_voxelmap* m, const int32_t* keys_xyz, size_t n, float* normals,
                                         float* centroids, uint8_t* present);
/* GetPointCloud: L0 centroids in L0 iteration order. */
size_t       lo_voxelmap_get_l0(const lo_voxelmap* m, float* xyz, size_t cap);
/* Upload the map's surfels to an ICP context (lo_map_set_surfels). */
int          lo_map_set_from_voxelmap(lo_ctx* ctx, const lo_voxelmap* m);
/* Bring the context's device surfel table up to date with the map after UpdateVoxelMap (Estimator.cpp:457): when the
 * table was last synced from this map, only the L1 voxels changed since then are patched in place
 * (lo_map_patch_surfels); otherwise (first sync, another map, KDTree mode, table full) the whole map is uploaded.
 * patched (nullable): the number of patched voxels, or -1 after a full upload. */
int          lo_map_sync_voxelmap(lo_ctx* ctx, const lo_voxelmap* m, int* patched);

/* FastVoxelFilter::filter(input, output, stride): returns the number of output points (<= n). */
size_t       lo_voxel_filter(const float* in_xyz, size_t n, float voxel_size, int stride, float* out_xyz);

/* ---- device-resident map ----
 * The same UpdateVoxelMap / AddPoint / radius prune / planarity erase / ApplyTransformAndRehash as lo_voxelmap_*,
 * kept in HBM next to an ICP context (surfel mode) whose surfel table it maintains in place: every update is ten
 * kernel launches on the context's stream and no host work, and the containers (L0 / L1 order, children order,
 * centroids, surfels) equal the host map's bit for bit.  Capacities are fixed at creation (max_l0 L0 voxels,
 * max_l0 / 2 L1 voxels, max_points per update); an overflow or a key beyond +-2^20 sets an error bit reported by
 * lo_devmap_counts / lo_devmap_status.  hierarchy_factor 1 or 3.  Destroy the map before its context.  The map
 * follows the context's stream: after lo_set_stream its launches go to the new stream. */
typedef struct lo_devmap lo_devmap;
lo_devmap*  lo_devmap_create(lo_ctx* ctx, float voxel_size, int hierarchy_factor, float planarity_threshold,
                             size_t max_l0, size_t max_points, int* err);
void        lo_devmap_destroy(lo_devmap* m);
const char* lo_devmap_last_error(const lo_devmap* m);
/* UpdateVoxelMap(cloud, sensor, max_distance, is_keyframe): world_xyz on the host (on_device = 0, copied) or a device
 * pointer (on_device = 1, read by the kernels, valid until they ran) */
int         lo_devmap_update(lo_devmap* m, const float* world_xyz, size_t n, int on_device, const double sensor[3],
                             double max_distance, int is_keyframe);
/* the context's last device-filtered scan moved to the world frame by T (util::transform_point_cloud) and inserted,
 * sensor = T's translation: create_keyframe's update (Estimator.cpp:370-530) without the scan leaving the device */
int         lo_devmap_update_from_scan(lo_devmap* m, const float T[12], double max_distance);
/* ApplyTransformAndRehash(T) (VoxelMap.cpp:264-302) + RecomputeAllSurfels (:304-366) */
int         lo_devmap_apply_transform(lo_devmap* m, const float T[12]);
/* out = {L0 voxels, L1 voxels, surfels, error bits}; syncs the stream.  LO_ERR_CAPACITY when error bits are set. */
int         lo_devmap_counts(lo_devmap* m, size_t out[4]);
/* the error bits only (one 64-byte copy; syncs the stream): LO_OK, or LO_ERR_CAPACITY with lo_devmap_last_error set
 * when an update overflowed a capacity or met a key beyond +-2^20 (the update aborted, the map is stale) */
int         lo_devmap_status(lo_devmap* m);
/* the same check without a stream sync: _async enqueues the copy of the error bits (pinned memory + an event) behind
 * the work enqueued so far; _poll returns LO_ERR_CAPACITY once that copy has landed and shows error bits, else LO_OK
 * (also while it is still in flight).  The frame loop enqueues after every keyframe's update and polls after each
 * frame's synchronous ICP, so an aborted update is reported at the first frame tracked after it. */
int         lo_devmap_status_async(lo_devmap* m);
/* KDTree-mode context (use_surfel_correspondence = 0): RebuildKdTree (VoxelMap.cpp:420-438) on the device -- the
 * context's correspondence grid rebuilt from the map's L0 centroids in L0 (GetPointCloud) order, equal to
 * lo_map_set_points on the same points; one small readback (count, bounds) per call.  Distance ties that the
 * reference's kd visit order would decide re-run the scan with that order (lo_kd_reruns). */
int         lo_devmap_sync_points(lo_devmap* m);
int         lo_devmap_status_poll(lo_devmap* m);
/* the containers in their order (tests / GetPointCloud): L0 keys, centroids, point counts; L1 keys, surfel flag,
 * normal, centroid, planarity, child count and children keys (27 per voxel) */
size_t      lo_devmap_get_l0(lo_devmap* m, int32_t* keys, float* xyz, int32_t* point_counts, size_t cap);
size_t      lo_devmap_get_l1(lo_devmap* m, int32_t* keys, uint8_t* has_surfel, float* normals, float* centroids,
                             float* planarity, int32_t* child_counts, int32_t* children, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* LO_MAP_H */
