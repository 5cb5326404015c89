/* lo_odometry.h — the frame loop around the ICP step (the hot path's caller), MI355X device path.
 *
 * Replaces Estimator::process_frame (src/processing/Estimator.cpp:115-233) for odometry without loop
 * closure / PGO (out of scope, off in all parity runs):
 *   preprocess_frame (:561-589)            -> device FastVoxelFilter (lo_icp_optimize_raw)
 *   first frame (:235-269)                 -> pose = initial pose, create_keyframe
 *   guess = prev_pose * velocity (:154)    -> SE3f product with SO3 re-projection (MathUtils.h:144-147)
 *   estimate_motion_dual_frame (:271-320) -> lo_icp_optimize_raw on the device map; failure keeps the guess
 *   velocity = prev^-1 * pose (:177)
 *   should_create_keyframe (:349-368)      -> |dt| > keyframe_distance or |Log(R_kf^-1 R)| > keyframe_rotation
 *   create_keyframe (:370-530)             -> VoxelMap::UpdateVoxelMap(world cloud, position, 1.2 * max_range):
 *                                             surfel mode: the device-resident map (lo_devmap_update_from_scan,
 *                                             lo_map.h), which patches the context's table in place -- ten kernel
 *                                             launches, no host sync (LO_HOST_MAP=1: the host map + patch sync);
 *                                             KDTree mode: the host map + RebuildKdTree upload
 */
#ifndef LO_ODOMETRY_H
#define LO_ODOMETRY_H

#include <stddef.h>

#include "lo_icp.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    lo_config icp;                 /* ICP + PKO + map geometry (voxel_size = map voxel, hierarchy_factor) */
    int    point_stride;           /* point_cloud.point_stride: 8 (kitti.yaml:18) */
    float  filter_voxel_size;      /* point_cloud.voxel_size: 0.5 (kitti.yaml:17) */
    double max_range;              /* point_cloud.max_range: 100 (kitti.yaml:20); map radius = 1.2 x */
    double keyframe_distance;      /* estimator.keyframe_distance_threshold: 1.0 m (kitti.yaml:55) */
    double keyframe_rotation;      /* estimator.keyframe_rotation_threshold: 0.3 rad (kitti.yaml:56) */
    float  planarity_threshold;    /* surfel planarity: 0.1 (kitti.yaml:22) */
} lo_odom_config;

typedef struct {
    int    status;                 /* LO_OK, or LO_INSUFFICIENT when ICP failed and the guess was kept */
    int    keyframe;               /* 1 if this frame became a keyframe (map updated) */
    int    icp_iterations;
    int    n_filtered;             /* feature cloud size */
    int    n_corr;
    double device_ms;              /* preprocessing + ICP on the device (HIP events) */
    double map_ms;                 /* keyframe map update (host wall time: enqueue only with the device map), 0 otherwise */
} lo_odom_frame;

typedef struct lo_odometry lo_odometry;

void          lo_odom_config_default_kitti(lo_odom_config* cfg);
/* The device map holds up to 2^21 L0 voxels (LO_DEVMAP_MAX_L0 in the environment overrides it).  An update that
 * overflows a capacity aborts and sets the map's error bits; lo_odom_process reports it (LO_ERR_CAPACITY) at the first
 * frame after that keyframe, read without a stream sync (lo_devmap_status_async / _poll). */
lo_odometry*  lo_odom_create(const lo_odom_config* cfg, int device, int* err);
void          lo_odom_destroy(lo_odometry* o);
const char*   lo_odom_last_error(const lo_odometry* o);
/* Pose of the first frame (LidarFrame::get_initial_pose); identity by default. */
int           lo_odom_set_initial_pose(lo_odometry* o, const float T[12]);
/* The frame loop's ICP arithmetic mode (lo_set_exact on its context): 1 = reference-exact, the default; 0 = the
 * opt-in fast mode (not parity-safe, see lo_set_exact).  Feature clouds whose bound ceil(n_raw / point_stride) exceeds
 * 16384 take the exact mode's device radix-sort path for the iteration-0 scale (slower, same bits). */
int           lo_odom_set_exact(lo_odometry* o, int enable);
/* One raw scan (AoS float3, host memory) -> its world pose (row-major 3x4).  Returns LO_OK / LO_INSUFFICIENT
 * (the guess was kept, as :304-307) or a negative error. */
int           lo_odom_process(lo_odometry* o, const float* raw_xyz, size_t n, float T_out[12], lo_odom_frame* info);
/* Wait for the last keyframe's map update and report its status: LO_ERR_CAPACITY if it overflowed (an overflow at the
 * final keyframe of a run is otherwise never read, since no later frame polls it).  Call before trusting the map after
 * the last frame; lo_odom_destroy does not report. */
int           lo_odom_flush(lo_odometry* o);
size_t        lo_odom_keyframe_count(const lo_odometry* o);
size_t        lo_odom_map_surfels(const lo_odometry* o);

#ifdef __cplusplus
}
#endif

#endif
