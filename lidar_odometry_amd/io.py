"""On-disk formats either side of the ICP step, backed by the C++ in liblo_icp.so
(lo_io.cpp): KITTI velodyne .bin, PLY point clouds, KITTI-format trajectories (camera frame)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._lib import lib


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _path(p) -> bytes:
    return os.fsencode(os.fspath(p))


def _check(n, path):
    if n < 0:
        raise OSError(f"cannot read {path} (code {n})")
    return n


def load_kitti_bin(path) -> np.ndarray:
    """util::load_kitti_binary (PointCloudUtils.cpp:18-65) -> (N, 3) float32."""
    n = _check(lib().lo_load_kitti_bin(_path(path), None, 0), path)
    out = np.zeros((max(n, 1), 3), np.float32)
    k = _check(lib().lo_load_kitti_bin(_path(path), _fp(out), n), path)
    return out[:k]


def load_ply(path) -> np.ndarray:
    """PLYPlayer::load_ply_point_cloud (ply_player.cpp:267-461) -> (N, 3) float32 (empty if no x/y/z)."""
    n = _check(lib().lo_load_ply(_path(path), None, 0), path)
    out = np.zeros((max(n, 1), 3), np.float32)
    k = _check(lib().lo_load_ply(_path(path), _fp(out), n), path)
    return out[:k]


def kitti_pose_line(pose) -> str:
    """KittiPlayer::pose_to_kitti_string: LiDAR pose (3x4 / 4x4) -> one KITTI camera-frame line."""
    p = np.ascontiguousarray(np.asarray(pose, np.float32)[:3, :4].reshape(12))
    buf = C.create_string_buffer(512)
    n = lib().lo_kitti_pose_line(_fp(p), buf, 512)
    if n < 0:
        raise ValueError("pose line")
    return buf.value.decode()


def save_trajectory_kitti(path, poses) -> None:
    """KittiPlayer::save_trajectory_kitti_format: one line per pose."""
    P = np.ascontiguousarray(np.stack([np.asarray(T, np.float32)[:3, :4] for T in poses]).reshape(-1, 12))
    rc = lib().lo_save_trajectory_kitti(_path(path), _fp(P), len(P))
    if rc != 0:
        raise OSError(f"cannot write {path} (code {rc})")


def load_trajectory_kitti(path) -> np.ndarray:
    """Read a KITTI trajectory file back to LiDAR-frame (N, 4, 4) poses (inverse of the camera-frame change)."""
    A = np.array([[0, -1, 0, 0], [0, 0, -1, 0], [1, 0, 0, 0], [0, 0, 0, 1]], np.float64)
    rows = np.loadtxt(path, ndmin=2).reshape(-1, 3, 4)
    out = np.tile(np.eye(4), (len(rows), 1, 1))
    out[:, :3, :4] = rows
    return np.einsum("ij,njk,kl->nil", A.T, out, A)
