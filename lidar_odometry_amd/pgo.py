"""Pose-graph optimisation: ctypes mirror of the reference's ``lidar_slam::optimization::PoseGraphOptimizer``
(src/optimization/PoseGraphOptimizer.h:86-210) over ``include/lo_pgo.h``.

Same method names, argument meaning and defaults; poses are 3x4 or 4x4 float arrays (the reference's SE3f) and come
back as 4x4 float32.  Host C++ (``csrc/lo_pgo.cpp``): batch Gauss-Newton on the keyframe graph with an envelope
LDL^T.  Parity unpinned (the reference's Eigen SimplicialLDLT / JacobiSVD are absent from this image).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import lib


def _pose12(T) -> np.ndarray:
    a = np.asarray(T, dtype=np.float32)
    if a.shape == (4, 4):
        a = a[:3]
    return np.ascontiguousarray(a.reshape(12), dtype=np.float32)


def _fp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _mat44(p12: np.ndarray) -> np.ndarray:
    T = np.eye(4, dtype=np.float32)
    T[:3] = p12.reshape(3, 4)
    return T


class PoseGraphOptimizer:
    def __init__(self):
        self._L = lib()
        self._h = self._L.lo_pgo_create()
        self.last_converged: bool | None = None      # the GN result the reference only logs (:275-280)
        self.last_iterations = 0
        self.last_ms = 0.0

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            self._h = None
            self._L.lo_pgo_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_first_keyframe(self, keyframe_id: int, pose) -> bool:
        p = _pose12(pose)
        return self._L.lo_pgo_add_first_keyframe(self._h, int(keyframe_id), _fp(p)) == 1

    def add_keyframe_with_odom(self, prev_keyframe_id: int, curr_keyframe_id: int, curr_pose, relative_pose,
                               odom_trans_noise: float = 0.1, odom_rot_noise: float = 0.1) -> bool:
        c, r = _pose12(curr_pose), _pose12(relative_pose)
        return self._L.lo_pgo_add_keyframe_with_odom(self._h, int(prev_keyframe_id), int(curr_keyframe_id), _fp(c),
                                                     _fp(r), float(odom_trans_noise), float(odom_rot_noise)) == 1

    def add_loop_and_optimize(self, from_keyframe_id: int, to_keyframe_id: int, relative_pose,
                              loop_trans_noise: float = 0.05, loop_rot_noise: float = 0.05) -> bool:
        r = _pose12(relative_pose)
        conv, its, ms = C.c_int(0), C.c_int(0), C.c_double(0.0)
        ok = self._L.lo_pgo_add_loop_and_optimize(self._h, int(from_keyframe_id), int(to_keyframe_id), _fp(r),
                                                  float(loop_trans_noise), float(loop_rot_noise), C.byref(conv),
                                                  C.byref(its), C.byref(ms)) == 1
        if ok:
            self.last_converged, self.last_iterations, self.last_ms = bool(conv.value), its.value, ms.value
        return ok

    def get_optimized_pose(self, keyframe_id: int):
        """(found, 4x4 pose) -- the reference's bool + out-parameter."""
        out = np.zeros(12, np.float32)
        ok = self._L.lo_pgo_get_optimized_pose(self._h, int(keyframe_id), _fp(out)) == 1
        return ok, (_mat44(out) if ok else None)

    def get_all_optimized_poses(self) -> dict:
        n = self.get_keyframe_count()
        ids = np.zeros(max(n, 1), np.int32)
        poses = np.zeros((max(n, 1), 12), np.float32)
        k = self._L.lo_pgo_get_all_optimized_poses(self._h, ids.ctypes.data_as(C.POINTER(C.c_int)), _fp(poses), n)
        return {int(ids[i]): _mat44(poses[i]) for i in range(k)}

    def has_keyframe(self, keyframe_id: int) -> bool:
        return self._L.lo_pgo_has_keyframe(self._h, int(keyframe_id)) == 1

    def get_keyframe_count(self) -> int:
        return int(self._L.lo_pgo_keyframe_count(self._h))

    def get_loop_closure_count(self) -> int:
        return int(self._L.lo_pgo_loop_closure_count(self._h))

    def clear(self):
        self._L.lo_pgo_clear(self._h)
