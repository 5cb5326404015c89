"""Map side of the product: ``VoxelMap`` (2-level voxel/surfel map) and ``voxel_filter``
(FastVoxelFilter) over the host C ABI in ``include/lo_map.h`` (``liblo_icp.so``).

``VoxelMap`` mirrors map::VoxelMap's build interface (src/database/VoxelMap.h:186-271):
``UpdateVoxelMap`` -> :meth:`update`, ``GetPointCloud`` -> :meth:`l0_cloud`, surfels -> :meth:`surfels`.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import lib


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class VoxelMap:
    def __init__(self, voxel_size: float = 0.5, hierarchy_factor: int = 3, planarity_threshold: float = 0.1,
                 compute_surfels: bool = True):
        self._L = lib()
        self._h = self._L.lo_voxelmap_create(voxel_size, hierarchy_factor, planarity_threshold, int(compute_surfels))
        if not self._h:
            raise ValueError("invalid VoxelMap parameters (voxel_size > 0, odd hierarchy_factor)")
        self.voxel_size = voxel_size
        self.hierarchy_factor = hierarchy_factor
        self.revision = 0

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            self._h = None
            self._L.lo_voxelmap_destroy(h)

    def __del__(self):
        # at interpreter teardown module globals (lib, os) may already be None: the handle keeps its own
        # reference to the loaded library, and a destructor never raises
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def update(self, world_points, sensor_position, max_distance: float, is_keyframe: bool = True):
        """VoxelMap::UpdateVoxelMap (VoxelMap.cpp:128-262)."""
        p = np.ascontiguousarray(world_points, dtype=np.float32).reshape(-1, 3)
        s = np.ascontiguousarray(sensor_position, dtype=np.float64).reshape(3)
        rc = lib().lo_voxelmap_update(self._h, _f(p), len(p), s.ctypes.data_as(C.POINTER(C.c_double)),
                                      float(max_distance), int(is_keyframe))
        if rc < 0:
            raise RuntimeError(f"lo_voxelmap_update failed ({rc})")
        self.revision += 1

    def set_device_fit(self, enable: bool = True):
        """Defer the surfel refits of update() to the next lo_map_sync_voxelmap of a context mirroring this map
        (k_surfel_fit on the device); bit-identical to host fits (include/lo_map.h)."""
        rc = lib().lo_voxelmap_set_device_fit(self._h, int(bool(enable)))
        if rc < 0:
            raise RuntimeError(f"lo_voxelmap_set_device_fit failed ({rc})")

    def apply_transform(self, T):
        """VoxelMap::ApplyTransformAndRehash (VoxelMap.cpp:264-302): T = row-major 3x4 (or 4x4) correction."""
        t = np.ascontiguousarray(np.asarray(T, np.float32)[:3, :] if np.asarray(T).ndim == 2 else
                                 np.asarray(T, np.float32).reshape(12)).reshape(12)
        rc = lib().lo_voxelmap_apply_transform(self._h, _f(t))
        if rc < 0:
            raise RuntimeError(f"lo_voxelmap_apply_transform failed ({rc})")
        self.revision += 1

    def l0_count(self) -> int:
        return int(lib().lo_voxelmap_l0_count(self._h))

    def l1_count(self) -> int:
        return int(lib().lo_voxelmap_l1_count(self._h))

    def surfel_count(self) -> int:
        return int(lib().lo_voxelmap_surfel_count(self._h))

    def surfels(self):
        """(keys int32 [m,3], normals [m,3], centroids [m,3], planarity [m]) in L1 iteration order."""
        m = self.surfel_count()
        k = np.zeros((max(m, 1), 3), np.int32)
        n = np.zeros((max(m, 1), 3), np.float32)
        c = np.zeros((max(m, 1), 3), np.float32)
        pl = np.zeros(max(m, 1), np.float32)
        got = lib().lo_voxelmap_get_surfels(self._h, k.ctypes.data_as(C.POINTER(C.c_int32)), _f(n), _f(c), _f(pl), m)
        return k[:got], n[:got], c[:got], pl[:got]

    def l0_cloud(self) -> np.ndarray:
        """VoxelMap::GetPointCloud (VoxelMap.cpp:388-403)."""
        m = self.l0_count()
        out = np.zeros((max(m, 1), 3), np.float32)
        got = lib().lo_voxelmap_get_l0(self._h, _f(out), m)
        return out[:got]


def voxel_filter(points, voxel_size: float, stride: int = 1) -> np.ndarray:
    """FastVoxelFilter::filter (VoxelMap.h:73-104): stride + Morton-keyed voxel centroids, first-occurrence order."""
    p = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
    out = np.zeros_like(p)
    n = lib().lo_voxel_filter(_f(p), len(p), float(voxel_size), int(stride), _f(out))
    return out[:n].copy()
