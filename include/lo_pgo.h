/*
 * lo_pgo.h — pose-graph optimisation C ABI (second half): the reference's
 * lidar_slam::optimization::PoseGraphOptimizer (src/optimization/PoseGraphOptimizer.h:86-210,
 * PoseGraphOptimizer.cpp:162-624) restated in host C++.  Same graph (one tight prior on the first keyframe,
 * odometry and loop-closure BetweenFactors with diagonal information), same batch Gauss-Newton (<= 10 iterations,
 * ||dx|| < 1e-6, T <- T Exp(dx) in GTSAM [rot, trans] order, every pose re-projected onto SO(3) through the SVD as
 * SE3d::FromMatrix does), the normal equations solved by a sparse LDL^T.
 *
 * Parity unpinned: the reference solves with Eigen::SimplicialLDLT (AMD ordering) and projects with
 * Eigen::JacobiSVD<Matrix3d>; Eigen is absent from this image, so the restatement is checked against an independent
 * dense numpy Gauss-Newton of the same equations and against pose graphs with a known optimum (tests/test_pgo.py),
 * not against the reference's own output.
 *
 * Poses are row-major 3x4 float (R | t), the reference's SE3f.  Functions returning int return 1 / 0 where the
 * reference returns bool, LO_ERR_ARG (< 0) for a null handle or pointer.
 */
#ifndef LO_PGO_H
#define LO_PGO_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lo_pgo lo_pgo;

lo_pgo* lo_pgo_create(void);
void    lo_pgo_destroy(lo_pgo* p);
/* add_first_keyframe (PoseGraphOptimizer.cpp:175-197): prior with sigma 1e-4 (rot and trans); 0 if not empty */
int     lo_pgo_add_first_keyframe(lo_pgo* p, int keyframe_id, const float pose[12]);
/* add_keyframe_with_odom (:199-244): BetweenFactor(prev, curr, relative) with the given sigmas, or a loose prior
 * (trans 0.5, rot 0.1) when prev is unknown; an existing curr is a no-op returning 1 */
int     lo_pgo_add_keyframe_with_odom(lo_pgo* p, int prev_keyframe_id, int curr_keyframe_id, const float curr_pose[12],
                                      const float relative_pose[12], double odom_trans_noise, double odom_rot_noise);
/* add_loop_and_optimize (:246-283): BetweenFactor(from, to, relative), then optimize(10, 1e-6).  0 if either
 * keyframe is unknown.  converged / iterations / ms (nullable): the GN result the reference only logs. */
int     lo_pgo_add_loop_and_optimize(lo_pgo* p, int from_keyframe_id, int to_keyframe_id, const float relative_pose[12],
                                     double loop_trans_noise, double loop_rot_noise, int* converged, int* iterations,
                                     double* ms);
/* get_optimized_pose (:285-295) */
int     lo_pgo_get_optimized_pose(const lo_pgo* p, int keyframe_id, float pose[12]);
/* get_all_optimized_poses (:297-305): ascending keyframe id (std::map order); returns the count written (<= cap) */
size_t  lo_pgo_get_all_optimized_poses(const lo_pgo* p, int* ids, float* poses, size_t cap);
int     lo_pgo_has_keyframe(const lo_pgo* p, int keyframe_id);
size_t  lo_pgo_keyframe_count(const lo_pgo* p);
size_t  lo_pgo_loop_closure_count(const lo_pgo* p);
void    lo_pgo_clear(lo_pgo* p);

#ifdef __cplusplus
}
#endif

#endif /* LO_PGO_H */
