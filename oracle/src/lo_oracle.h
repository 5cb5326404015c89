/*
 * lo_oracle.h — C ABI of the CPU ORACLE (test infrastructure only).
 *
 * This library is a single-threaded CPU restatement of the reference ICP hot path
 * (SiarheiHerasiuta/lidar_odometry).  It is the parity checker for the HIP product
 * in lidar_odometry_amd/ and the `cpu_baseline` leg of bench.py.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  It is never
 * linked into or called by the product.
 *
 * Parity pinning: the PKO part (or_pko_*) is pinned against golden vectors produced by
 * the reference's own AdaptiveMEstimator.cpp compiled in place (oracle/ref/pko_golden.cpp,
 * fixtures in tests/golden/).  The Eigen-dependent parts (JacobiSVD, LDLT, SE3, VoxelMap,
 * correspondence search) are restated from the reference source and are
 * "parity unpinned" against reference binaries: Eigen is not installed in the container,
 * so the reference ICP cannot be built.
 */
#ifndef LO_ORACLE_H
#define LO_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* PKO configuration (AdaptiveMEstimatorConfig, AdaptiveMEstimator.h:24-41). */
typedef struct or_pko_cfg {
    double min_scale_factor;      /* 0.1  (config/kitti.yaml:43) */
    double max_scale_factor;      /* 10.0 */
    int    num_alpha_segments;    /* 100  */
    double truncated_threshold;   /* 10.0 */
    int    gmm_components;        /* 3    */
    int    gmm_sample_size;       /* 100  */
    int    kernel;                /* pko_kernel_type: 0 huber, 1 cauchy, 2 tukey, 3 welsch, 4 gemanMcClure, 5 pseudoHuber */
} or_pko_cfg;

/* ICP configuration (ICPConfig, IterativeClosestPointOptimizer.h:55-76 as wired by Estimator.cpp:62-70). */
typedef struct or_icp_cfg {
    int    max_iterations;              /* 4 */
    double translation_tolerance;       /* 0.005 */
    double rotation_tolerance;          /* 0.005 */
    double max_correspondence_distance; /* 1.0 */
    int    min_correspondence_points;   /* 10 */
    int    use_robust_loss;             /* 1 */
    double robust_loss_delta;           /* 0.1 (only without PKO) */
    int    use_pko;                     /* 1 (use_adaptive_m_estimator) */
    int    loss_cauchy;                 /* 0 = huber weight (loss_type never parsed -> "huber") */
    or_pko_cfg pko;
} or_icp_cfg;

/* One executed GN iteration. */
typedef struct or_iter_log {
    float  pose[12];      /* row-major [R|t] AFTER this iteration's update */
    int    n_corr;        /* correspondences found */
    double scale;         /* residual normalisation scale (iteration-0 value) */
    double alpha;         /* PKO delta */
    float  cost;          /* sum w r^2 (fp32, sequential) */
    float  H[21];         /* upper triangle of H, row-major (0,0),(0,1)..(0,5),(1,1).. */
    float  g[6];
    float  delta[6];      /* [dt, dw] */
} or_iter_log;

/* ---- PKO (AdaptiveMEstimator) ---- */
double or_pko_scale_factor(const or_pko_cfg* cfg, const double* residuals, int n,
                           double* gmm_out /* 3*comps: weights, means, variances; nullable */);
/* First k entries of std::shuffle(iota(n), std::mt19937(42)) (AdaptiveMEstimator.cpp:319-323). */
void   or_shuffle_prefix(int n, int k, int* out);
/* The two k-means seed draws uniform_int_distribution<>(0, m-1) of a fresh mt19937(42) (:336-345). */
void   or_kmeans_seed_draws(int m, int count, int* out);
/* Alpha grid and partition functions (initialize_pko, :218-241). out arrays of size segs+1. */
void   or_pko_tables(const or_pko_cfg* cfg, double* alphas, double* Z);

/* ---- SO3/SE3 + linear algebra (MathUtils.cpp) ---- */
void   or_se3_inverse(const float A[12], float out[12]);
void   or_keyframe_metrics(const float kf[12], const float pose[12], double out[2]);
void   or_se3_compose(const float A[12], const float B[12], float out[12]);   /* SE3::operator* */
void   or_so3_exp(const float w[3], float R[9]);                             /* SO3::Exp (incl. SVD ctor) */
void   or_so3_normalize(const float Rin[9], float Rout[9]);                   /* SO3(Matrix3f) */
int    or_jacobi_svd3(const float A[9], float U[9], float S[3], float V[9]);  /* JacobiSVD<Matrix3f> */
void   or_ldlt6_solve(const float H[36], const float b[6], float x[6]);       /* H.ldlt().solve(b) */

/* ---- Voxel map (VoxelMap.cpp) ---- */
void*  or_map_create(float voxel_size, int hierarchy_factor, float planarity_threshold, int compute_surfels);
void   or_map_destroy(void* m);
void   or_map_update(void* m, const float* xyz, int n, const double sensor[3], double max_distance, int is_keyframe);
void   or_map_apply_transform(void* m, const float T[12]);
/* container-operation trace of the map (7 int32 per record, see VoxelMap::trace) and the iteration orders */
void   or_map_trace(void* m, int enable);
size_t or_map_trace_get(const void* m, int32_t* out, size_t cap);
size_t or_map_orders(const void* m, int32_t* l0, int32_t* l1, int32_t* child_cnt, int32_t* children, size_t cap);
int    or_map_l0_count(void* m);
int    or_map_l1_count(void* m);
int    or_map_surfel_count(void* m);
/* Surfels in L1 iteration order: keys int32 x3, normal x3, centroid x3, planarity. */
int    or_map_get_surfels(void* m, int32_t* keys, float* normals, float* centroids, float* planarity, int cap);
/* GetPointCloud: L0 centroids in L0 iteration order. */
int    or_map_get_l0(void* m, float* xyz, int cap);
int    or_map_lookup(void* m, const float p[3], float n[3], float c[3]);

/* ---- FastVoxelFilter (VoxelMap.h:73-104) ---- */
int    or_voxel_filter(const float* in, int n, float voxel_size, int stride, float* out);

/* ---- transform_point_cloud (PointCloudUtils.cpp:102-125) ---- */
void   or_transform_points(const float* in, int n, const float T[12], float* out);

/* ---- ICP (IterativeClosestPointOptimizer.cpp) ---- */
/* find_correspondences at pose T: per input point valid flag and fp64 residual (0 if invalid). */
int    or_find_correspondences(void* map, const float* pts, int n, const float T[12],
                               double max_corr_dist, uint8_t* valid, double* residual);
/* find_correspondences_kdtree at pose T (brute-force exact 5-NN over L0 centroids). */
void   or_set_kdtree_search(int use_tree);   /* 1: kd-tree (default), 0: exhaustive scan in nanoflann's order */
/* util::KdTree::nearestKSearch(q, 5) over `cloud` for every query (nanoflann restated); idx -1 / dist inf past found */
void   or_kdtree_knn5(const float* cloud, int m, const float* q, int nq, int use_tree, int* idx, float* dist, int* found);
int    or_find_correspondences_kdtree(void* map, const float* pts, int n, const float T[12],
                                      double max_corr_dist, uint8_t* valid, double* residual,
                                      float* normal_out /* nullable, n*3 */, float* target_out /* nullable */);
/* optimize(): returns 1 on success, 0 on insufficient correspondences.  use_kdtree selects
   find_correspondences_kdtree.  logs: max_iterations entries (nullable). */
int    or_icp_optimize(void* map, const float* pts, int n, const float T_init[12], float T_out[12],
                       const or_icp_cfg* cfg, int use_kdtree, or_iter_log* logs, int* iterations);
/* optimize_loop (IterativeClosestPointOptimizer.cpp:40-251): returns 1 = success (converged and inlier ratio >= 0.5).
 * T_rel / inlier_ratio are written only when converged (*converged = 1); logs receives up to max_logs iterations. */
int    or_icp_optimize_loop(const float* curr, int n_curr, const float T_curr[12], const float* matched, int n_matched,
                            const float T_matched[12], const or_icp_cfg* cfg, float T_rel[12], float* inlier_ratio,
                            or_iter_log* logs, int max_logs, int* iterations, int* converged);
/* Build the weighted normal equations of one iteration for given pose / scale / delta. */
int    or_build_normal_equations(void* map, const float* pts, int n, const float T[12],
                                 const or_icp_cfg* cfg, double scale, double delta,
                                 float H[36], float g[6], float* cost);

#ifdef __cplusplus
}
#endif
#endif
