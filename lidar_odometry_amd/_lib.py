"""ctypes binding of ``liblo_icp.so`` (the C ABI in ``include/lo_icp.h``).

The shared library is built in-tree by ``make -C lidar_odometry_amd/csrc`` (``__graft_entry__.build()``).
There is no CPU fallback: if the library or a HIP device is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LO_ICP_LIB") or os.path.join(_HERE, "liblo_icp.so")

LO_OK = 0
LO_INSUFFICIENT = 1
LO_ERR_ARG = -1
LO_ERR_HIP = -2
LO_ERR_CAPACITY = -3
LO_ERR_STATE = -4
LO_ERR_PIPELINE = -5
LO_MAX_ITERS = 64

# Every symbol include/lo_icp.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "lo_config_default_kitti", "lo_config_default_mid360", "lo_pko_kernel_from_name", "lo_create", "lo_destroy", "lo_last_error",
    "lo_device", "lo_get_config", "lo_map_set_surfels", "lo_map_surfel_count", "lo_map_set_points",
    "lo_map_point_count", "lo_icp_optimize", "lo_icp_optimize_raw_async", "lo_icp_optimize_raw", "lo_filtered_points",
    "lo_voxel_filter_gpu", "lo_icp_optimize_async", "lo_icp_optimize_loop", "lo_host_alloc", "lo_host_free",
    "lo_icp_result", "lo_sync", "lo_stream", "lo_set_stream", "lo_set_exact", "lo_set_pipeline", "lo_pipeline_status", "lo_set_pko_groups", "lo_update_config", "lo_map_sync_surfels", "lo_set_stage_timing", "lo_stage_time", "lo_pko_em_stats", "lo_icp_export_pose", "lo_bench_kernel", "lo_bench_correspond_rr", "lo_find_correspondences", "lo_knn_search", "lo_pko_scale_factor",
    "lo_build_normal_equations", "lo_pko_sample_indices", "lo_pko_sample_indices_host", "lo_debug_counters", "lo_debug_counters_ex", "lo_stage_span", "lo_seq_sum_f64", "lo_seq_sum_f32",
    "lo_batch_create", "lo_batch_destroy", "lo_batch_last_error", "lo_batch_size", "lo_batch_optimize_async",
    "lo_batch_result", "lo_batch_optimize", "lo_batch_bench_correspond",
    # include/lo_map.h
    "lo_voxelmap_create", "lo_voxelmap_destroy", "lo_voxelmap_update", "lo_voxelmap_l0_count",
    "lo_voxelmap_l1_count", "lo_voxelmap_surfel_count", "lo_voxelmap_get_surfels", "lo_voxelmap_get_l0", "lo_voxelmap_changed_l1", "lo_voxelmap_surfel_at", "lo_voxelmap_surfels_at_keys",
    "lo_map_set_from_voxelmap", "lo_map_sync_voxelmap", "lo_voxelmap_apply_transform", "lo_map_patch_surfels", "lo_voxel_filter",
    "lo_voxelmap_set_device_fit", "lo_devmap_create", "lo_devmap_destroy", "lo_devmap_last_error", "lo_devmap_update",
    "lo_devmap_update_from_scan", "lo_devmap_apply_transform", "lo_devmap_counts", "lo_devmap_status", "lo_devmap_status_async", "lo_devmap_status_poll", "lo_devmap_sync_points", "lo_kd_reruns", "lo_devmap_get_l0", "lo_devmap_get_l1",
    # include/lo_odometry.h
    "lo_odom_config_default_kitti", "lo_odom_create", "lo_odom_destroy", "lo_odom_last_error", "lo_odom_set_initial_pose",
    "lo_odom_process", "lo_odom_keyframe_count", "lo_odom_map_surfels", "lo_odom_set_exact", "lo_odom_flush",
    # include/lo_io.h
    "lo_load_kitti_bin", "lo_load_ply", "lo_kitti_pose_line", "lo_save_trajectory_kitti",
    # include/lo_pgo.h
    "lo_pgo_create", "lo_pgo_destroy", "lo_pgo_add_first_keyframe", "lo_pgo_add_keyframe_with_odom",
    "lo_pgo_add_loop_and_optimize", "lo_pgo_get_optimized_pose", "lo_pgo_get_all_optimized_poses",
    "lo_pgo_has_keyframe", "lo_pgo_keyframe_count", "lo_pgo_loop_closure_count", "lo_pgo_clear",
)


class LoConfig(C.Structure):
    _fields_ = [
        ("max_iterations", C.c_int), ("translation_tolerance", C.c_double), ("rotation_tolerance", C.c_double),
        ("max_correspondence_distance", C.c_double), ("min_correspondence_points", C.c_int),
        ("use_robust_loss", C.c_int), ("robust_loss_delta", C.c_double), ("loss_cauchy", C.c_int),
        ("use_adaptive_m_estimator", C.c_int), ("min_scale_factor", C.c_double), ("max_scale_factor", C.c_double),
        ("num_alpha_segments", C.c_int), ("truncated_threshold", C.c_double), ("gmm_components", C.c_int),
        ("gmm_sample_size", C.c_int), ("pko_kernel", C.c_int), ("voxel_size", C.c_float),
        ("hierarchy_factor", C.c_int), ("use_surfel_correspondence", C.c_int), ("max_points", C.c_int),
    ]


class LoIterLog(C.Structure):
    _fields_ = [("pose", C.c_float * 12), ("n_corr", C.c_int), ("scale", C.c_double), ("alpha", C.c_double),
                ("cost", C.c_float), ("H", C.c_float * 21), ("g", C.c_float * 6), ("delta", C.c_float * 6)]


class LoStats(C.Structure):
    _fields_ = [("iterations", C.c_int), ("n_corr", C.c_int), ("status", C.c_int), ("converged", C.c_int),
                ("initial_cost", C.c_double), ("final_cost", C.c_double), ("gpu_ms", C.c_double)]


class LoBatchRec(C.Structure):
    _fields_ = [("pose", C.c_float * 12), ("status", C.c_int), ("iterations", C.c_int), ("n_corr", C.c_int),
                ("initial_cost", C.c_float), ("final_cost", C.c_float), ("pad", C.c_float), ("alpha", C.c_double)]


class LoOdomConfig(C.Structure):
    _fields_ = [("icp", LoConfig), ("point_stride", C.c_int), ("filter_voxel_size", C.c_float), ("max_range", C.c_double),
                ("keyframe_distance", C.c_double), ("keyframe_rotation", C.c_double), ("planarity_threshold", C.c_float)]


class LoOdomFrame(C.Structure):
    _fields_ = [("status", C.c_int), ("keyframe", C.c_int), ("icp_iterations", C.c_int), ("n_filtered", C.c_int),
                ("n_corr", C.c_int), ("device_ms", C.c_double), ("map_ms", C.c_double)]


_lib = None


def lib():
    """Load liblo_icp.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"HIP extension missing: {LIB_PATH}. Build it with `make -C lidar_odometry_amd/csrc` "
                           "(there is no CPU fallback).")
    L = C.CDLL(LIB_PATH)
    fp, dp, ip, u8p, vp = (C.POINTER(C.c_float), C.POINTER(C.c_double), C.POINTER(C.c_int32),
                           C.POINTER(C.c_uint8), C.c_void_p)
    L.lo_config_default_kitti.argtypes = [C.POINTER(LoConfig)]
    L.lo_config_default_mid360.argtypes = [C.POINTER(LoConfig)]
    L.lo_create.restype = vp
    L.lo_create.argtypes = [C.POINTER(LoConfig), C.c_int, C.POINTER(C.c_int)]
    L.lo_destroy.argtypes = [vp]
    L.lo_last_error.restype = C.c_char_p
    L.lo_last_error.argtypes = [vp]
    L.lo_device.argtypes = [vp]
    L.lo_map_set_surfels.argtypes = [vp, ip, fp, fp, C.c_size_t]
    L.lo_map_surfel_count.restype = C.c_size_t
    L.lo_map_surfel_count.argtypes = [vp]
    L.lo_map_set_points.restype = C.c_int
    L.lo_map_set_points.argtypes = [vp, C.POINTER(C.c_float), C.c_size_t]
    L.lo_map_point_count.restype = C.c_size_t
    L.lo_map_point_count.argtypes = [vp]
    L.lo_icp_optimize_raw_async.restype = C.c_int
    L.lo_icp_optimize_raw_async.argtypes = [vp, vp, C.c_size_t, C.c_int, C.c_float, fp]
    L.lo_icp_optimize_raw.restype = C.c_int
    L.lo_icp_optimize_raw.argtypes = [vp, fp, C.c_size_t, C.c_int, C.c_float, fp, fp, C.POINTER(LoIterLog),
                                      C.POINTER(LoStats)]
    L.lo_host_alloc.restype = vp
    L.lo_host_alloc.argtypes = [C.c_size_t]
    L.lo_host_free.restype = None
    L.lo_host_free.argtypes = [vp]
    L.lo_icp_optimize_loop.restype = C.c_int
    L.lo_icp_optimize_loop.argtypes = [vp, fp, C.c_size_t, fp, fp, C.c_size_t, fp, fp, fp, C.POINTER(LoIterLog),
                                       C.POINTER(LoStats)]
    L.lo_filtered_points.restype = C.c_longlong
    L.lo_filtered_points.argtypes = [vp, fp, C.c_size_t]
    L.lo_voxel_filter_gpu.restype = C.c_longlong
    L.lo_voxel_filter_gpu.argtypes = [vp, fp, C.c_size_t, C.c_float, C.c_int, fp, C.c_size_t]
    L.lo_odom_config_default_kitti.argtypes = [C.POINTER(LoOdomConfig)]
    L.lo_odom_create.restype = vp
    L.lo_odom_create.argtypes = [C.POINTER(LoOdomConfig), C.c_int, C.POINTER(C.c_int)]
    L.lo_odom_destroy.argtypes = [vp]
    L.lo_odom_last_error.restype = C.c_char_p
    L.lo_odom_last_error.argtypes = [vp]
    L.lo_odom_set_initial_pose.argtypes = [vp, fp]
    L.lo_odom_process.restype = C.c_int
    L.lo_odom_process.argtypes = [vp, fp, C.c_size_t, fp, C.POINTER(LoOdomFrame)]
    L.lo_odom_keyframe_count.restype = C.c_size_t
    L.lo_odom_keyframe_count.argtypes = [vp]
    L.lo_odom_map_surfels.restype = C.c_size_t
    L.lo_odom_map_surfels.argtypes = [vp]
    L.lo_odom_set_exact.argtypes = [vp, C.c_int]
    L.lo_odom_flush.restype = C.c_int
    L.lo_odom_flush.argtypes = [vp]
    L.lo_load_kitti_bin.restype = C.c_longlong
    L.lo_load_kitti_bin.argtypes = [C.c_char_p, fp, C.c_size_t]
    L.lo_load_ply.restype = C.c_longlong
    L.lo_load_ply.argtypes = [C.c_char_p, fp, C.c_size_t]
    L.lo_kitti_pose_line.restype = C.c_int
    L.lo_kitti_pose_line.argtypes = [fp, C.c_char_p, C.c_size_t]
    L.lo_save_trajectory_kitti.restype = C.c_int
    L.lo_save_trajectory_kitti.argtypes = [C.c_char_p, fp, C.c_size_t]
    L.lo_devmap_create.restype = vp
    L.lo_devmap_create.argtypes = [vp, C.c_float, C.c_int, C.c_float, C.c_size_t, C.c_size_t, C.POINTER(C.c_int)]
    L.lo_devmap_destroy.restype = None
    L.lo_devmap_destroy.argtypes = [vp]
    L.lo_devmap_last_error.restype = C.c_char_p
    L.lo_devmap_last_error.argtypes = [vp]
    L.lo_devmap_update.argtypes = [vp, vp, C.c_size_t, C.c_int, dp, C.c_double, C.c_int]
    L.lo_devmap_update_from_scan.argtypes = [vp, fp, C.c_double]
    L.lo_devmap_apply_transform.argtypes = [vp, fp]
    L.lo_devmap_counts.argtypes = [vp, C.POINTER(C.c_size_t)]
    L.lo_devmap_status.argtypes = [vp]
    L.lo_devmap_status_async.argtypes = [vp]
    L.lo_devmap_status_poll.argtypes = [vp]
    L.lo_devmap_sync_points.argtypes = [vp]
    L.lo_kd_reruns.argtypes = [vp]
    L.lo_devmap_get_l0.restype = C.c_size_t
    L.lo_devmap_get_l0.argtypes = [vp, ip, fp, ip, C.c_size_t]
    L.lo_devmap_get_l1.restype = C.c_size_t
    L.lo_devmap_get_l1.argtypes = [vp, ip, u8p, fp, fp, fp, ip, ip, C.c_size_t]
    L.lo_pgo_create.restype = vp
    L.lo_pgo_create.argtypes = []
    L.lo_pgo_destroy.restype = None
    L.lo_pgo_destroy.argtypes = [vp]
    L.lo_pgo_add_first_keyframe.argtypes = [vp, C.c_int, fp]
    L.lo_pgo_add_keyframe_with_odom.argtypes = [vp, C.c_int, C.c_int, fp, fp, C.c_double, C.c_double]
    L.lo_pgo_add_loop_and_optimize.argtypes = [vp, C.c_int, C.c_int, fp, C.c_double, C.c_double,
                                               C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_double)]
    L.lo_pgo_get_optimized_pose.argtypes = [vp, C.c_int, fp]
    L.lo_pgo_get_all_optimized_poses.restype = C.c_size_t
    L.lo_pgo_get_all_optimized_poses.argtypes = [vp, C.POINTER(C.c_int), fp, C.c_size_t]
    L.lo_pgo_has_keyframe.argtypes = [vp, C.c_int]
    L.lo_pgo_keyframe_count.restype = C.c_size_t
    L.lo_pgo_keyframe_count.argtypes = [vp]
    L.lo_pgo_loop_closure_count.restype = C.c_size_t
    L.lo_pgo_loop_closure_count.argtypes = [vp]
    L.lo_pgo_clear.restype = None
    L.lo_pgo_clear.argtypes = [vp]
    L.lo_get_config.restype = C.c_int
    L.lo_pko_kernel_from_name.restype = C.c_int
    L.lo_pko_kernel_from_name.argtypes = [C.c_char_p]
    L.lo_get_config.argtypes = [vp, C.POINTER(LoConfig)]
    L.lo_icp_optimize.argtypes = [vp, fp, C.c_size_t, fp, fp, C.POINTER(LoIterLog), C.POINTER(LoStats)]
    L.lo_icp_optimize_async.argtypes = [vp, C.c_void_p, C.c_size_t, fp]
    L.lo_icp_result.argtypes = [vp, fp, C.POINTER(LoIterLog), C.POINTER(LoStats)]
    L.lo_sync.argtypes = [vp]
    L.lo_stream.restype = vp
    L.lo_stream.argtypes = [vp]
    L.lo_set_stream.argtypes = [vp, vp]
    L.lo_set_exact.argtypes = [vp, C.c_int]
    L.lo_set_pipeline.argtypes = [vp, C.c_int, C.c_int]
    L.lo_set_stage_timing.argtypes = [vp, C.c_int]
    L.lo_stage_time.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_int)]
    L.lo_stage_span.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_int)]
    L.lo_pko_em_stats.argtypes = [vp, C.POINTER(C.c_ulonglong), C.c_int]
    L.lo_icp_export_pose.argtypes = [vp, vp]
    L.lo_bench_kernel.argtypes = [vp, vp, C.c_size_t, fp, C.c_double, C.c_double, C.c_int, C.c_int, fp]
    L.lo_bench_correspond_rr.argtypes = [C.POINTER(vp), C.POINTER(vp), C.POINTER(C.c_size_t), fp, C.c_int, C.c_int, fp]
    L.lo_find_correspondences.argtypes = [vp, fp, C.c_size_t, fp, u8p, dp]
    L.lo_knn_search.argtypes = [vp, fp, C.c_size_t, ip, fp]
    L.lo_pko_scale_factor.restype = C.c_double
    L.lo_pko_scale_factor.argtypes = [vp, dp, C.c_size_t, dp]
    L.lo_build_normal_equations.argtypes = [vp, fp, C.c_size_t, fp, C.c_double, C.c_double, dp, dp, dp]
    L.lo_pko_sample_indices.argtypes = [vp, C.c_size_t, ip]
    L.lo_pko_sample_indices_host.argtypes = [C.c_size_t, C.c_int, ip]
    L.lo_debug_counters.argtypes = [vp, C.POINTER(C.c_ulonglong)]
    L.lo_debug_counters_ex.argtypes = [vp, C.POINTER(C.c_ulonglong), C.c_int]
    L.lo_pipeline_status.argtypes = [vp, C.POINTER(C.c_int)]
    L.lo_set_pko_groups.argtypes = [vp, C.c_int]
    L.lo_update_config.argtypes = [vp, C.POINTER(LoConfig)]
    L.lo_map_sync_surfels.argtypes = [vp, C.POINTER(C.c_int32), C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_size_t,
                                      C.POINTER(C.c_int)]
    L.lo_seq_sum_f32.argtypes = [vp, C.POINTER(C.c_float), C.c_size_t, C.POINTER(C.c_float), C.POINTER(C.c_longlong)]
    L.lo_seq_sum_f64.argtypes = [vp, C.POINTER(C.c_double), C.c_size_t, C.c_int, C.POINTER(C.c_double),
                                 C.POINTER(C.c_longlong)]
    L.lo_batch_create.restype = vp
    L.lo_batch_create.argtypes = [C.POINTER(vp), C.c_int, C.POINTER(C.c_int)]
    L.lo_batch_destroy.restype = None
    L.lo_batch_destroy.argtypes = [vp]
    L.lo_batch_last_error.restype = C.c_char_p
    L.lo_batch_last_error.argtypes = [vp]
    L.lo_batch_size.argtypes = [vp]
    L.lo_batch_optimize_async.argtypes = [vp, C.POINTER(vp), C.POINTER(C.c_size_t), fp]
    L.lo_batch_result.argtypes = [vp, C.POINTER(LoBatchRec), dp]
    L.lo_batch_bench_correspond.argtypes = [vp, C.c_int, fp]
    L.lo_batch_optimize.argtypes = [vp, C.POINTER(vp), C.POINTER(C.c_size_t), fp, C.POINTER(LoBatchRec)]
    L.lo_voxelmap_create.restype = vp
    L.lo_voxelmap_create.argtypes = [C.c_float, C.c_int, C.c_float, C.c_int]
    L.lo_voxelmap_destroy.argtypes = [vp]
    L.lo_voxelmap_update.argtypes = [vp, fp, C.c_size_t, dp, C.c_double, C.c_int]
    for f in ("lo_voxelmap_l0_count", "lo_voxelmap_l1_count", "lo_voxelmap_surfel_count"):
        getattr(L, f).restype = C.c_size_t
        getattr(L, f).argtypes = [vp]
    L.lo_voxelmap_get_surfels.restype = C.c_size_t
    L.lo_voxelmap_get_surfels.argtypes = [vp, ip, fp, fp, fp, C.c_size_t]
    L.lo_voxelmap_changed_l1.restype = C.c_size_t
    L.lo_voxelmap_changed_l1.argtypes = [vp, ip, C.c_size_t]
    L.lo_voxelmap_surfel_at.restype = C.c_int
    L.lo_voxelmap_surfel_at.argtypes = [vp, fp, fp, fp]
    L.lo_voxelmap_surfels_at_keys.restype = C.c_size_t
    L.lo_voxelmap_surfels_at_keys.argtypes = [vp, ip, C.c_size_t, fp, fp, vp]
    L.lo_voxelmap_get_l0.restype = C.c_size_t
    L.lo_voxelmap_get_l0.argtypes = [vp, fp, C.c_size_t]
    L.lo_map_set_from_voxelmap.argtypes = [vp, vp]
    L.lo_map_sync_voxelmap.argtypes = [vp, vp, C.POINTER(C.c_int)]
    L.lo_voxelmap_apply_transform.argtypes = [vp, vp]
    L.lo_voxelmap_set_device_fit.argtypes = [vp, C.c_int]
    L.lo_map_patch_surfels.argtypes = [vp, vp, vp, vp, vp, C.c_size_t]
    L.lo_voxel_filter.restype = C.c_size_t
    L.lo_voxel_filter.argtypes = [fp, C.c_size_t, C.c_float, C.c_int, fp]
    _lib = L
    return L


def pinned_empty(shape, dtype=np.float32):
    """A numpy array in page-locked, device-accessible host memory (lo_host_alloc): raw scans placed in it are read
    by the device filter directly, without a staging copy.  The memory is released with the array."""
    dt = np.dtype(dtype)
    n = max(int(np.prod(shape)) * dt.itemsize, 1)
    ptr = lib().lo_host_alloc(n)
    if not ptr:
        raise MemoryError(f"lo_host_alloc({n}) failed")
    buf = (C.c_char * n).from_address(ptr)
    buf._release = weakref.finalize(buf, lib().lo_host_free, C.c_void_p(ptr))
    return np.frombuffer(buf, dtype=dt, count=int(np.prod(shape))).reshape(shape)
