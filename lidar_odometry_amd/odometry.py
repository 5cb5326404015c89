"""Frame loop around the ICP step (Estimator::process_frame without loop closure / PGO), C++ in liblo_icp.so
(lo_odometry.cpp, include/lo_odometry.h): device voxel filter + device GN ICP per frame, SE3f bookkeeping,
keyframe map updates."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import LoOdomConfig, LoOdomFrame, lib


@dataclass
class FrameInfo:
    status: int
    keyframe: bool
    icp_iterations: int
    n_filtered: int
    n_corr: int
    device_ms: float
    map_ms: float


class LidarOdometry:
    """One sensor stream on one GPU: process(raw_points) -> 3x4 world pose (config/kitti.yaml defaults)."""

    def __init__(self, device: int = 0, max_points: int = 1 << 17, use_surfel_correspondence: bool = True,
                 point_stride: int = 8, voxel_size: float = 0.5, map_voxel_size: float = 0.5, max_range: float = 100.0,
                 keyframe_distance: float = 1.0, keyframe_rotation: float = 0.3, initial_pose=None,
                 exact: bool = True):
        cfg = LoOdomConfig()
        lib().lo_odom_config_default_kitti(C.byref(cfg))
        cfg.icp.max_points = int(max_points)
        cfg.icp.use_surfel_correspondence = int(bool(use_surfel_correspondence))
        cfg.icp.voxel_size = float(map_voxel_size)
        cfg.point_stride = int(point_stride)
        cfg.filter_voxel_size = float(voxel_size)
        cfg.max_range = float(max_range)
        cfg.keyframe_distance = float(keyframe_distance)
        cfg.keyframe_rotation = float(keyframe_rotation)
        err = C.c_int(0)
        self._L = lib()
        self._o = self._L.lo_odom_create(C.byref(cfg), int(device), C.byref(err))
        if not self._o:
            raise RuntimeError(f"lo_odom_create failed (code {err.value}); is a HIP device present?")
        if initial_pose is not None:
            T = np.ascontiguousarray(np.asarray(initial_pose, np.float32)[:3, :4].reshape(12))
            lib().lo_odom_set_initial_pose(self._o, T.ctypes.data_as(C.POINTER(C.c_float)))
        # the ICP arithmetic mode: reference-exact (the library default, lo_set_exact) or the opt-in fast mode
        lib().lo_odom_set_exact(self._o, 1 if exact else 0)

    def close(self):
        h = getattr(self, "_o", None)
        if h:
            self._o = None
            self._L.lo_odom_destroy(h)

    def __del__(self):
        # at interpreter teardown module globals (lib, os) may already be None: the handle keeps its own
        # reference to the loaded library, and a destructor never raises
        try:
            self.close()
        except Exception:
            pass

    def process(self, raw_points):
        p = np.ascontiguousarray(raw_points, dtype=np.float32).reshape(-1, 3)
        T = np.zeros(12, np.float32)
        info = LoOdomFrame()
        rc = lib().lo_odom_process(self._o, p.ctypes.data_as(C.POINTER(C.c_float)), len(p),
                                   T.ctypes.data_as(C.POINTER(C.c_float)), C.byref(info))
        if rc < 0:
            raise RuntimeError(f"lo_odom_process error {rc}: {lib().lo_odom_last_error(self._o).decode()}")
        return T.reshape(3, 4), FrameInfo(info.status, bool(info.keyframe), info.icp_iterations, info.n_filtered,
                                          info.n_corr, info.device_ms, info.map_ms)

    def flush(self):
        """Wait for the last keyframe's map update; raise if it overflowed the device map (lo_odom_flush)."""
        rc = lib().lo_odom_flush(self._o)
        if rc < 0:
            raise RuntimeError(f"lo_odom_flush error {rc}: {lib().lo_odom_last_error(self._o).decode()}")

    @property
    def keyframes(self) -> int:
        return int(lib().lo_odom_keyframe_count(self._o))

    @property
    def map_surfels(self) -> int:
        return int(lib().lo_odom_map_surfels(self._o))


__all__ = ["LidarOdometry", "FrameInfo", "_lib"]
