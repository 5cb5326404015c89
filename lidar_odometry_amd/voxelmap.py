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

    def changed_l1(self) -> np.ndarray:
        """The L1 keys whose surfel the last update may have changed (lo_voxelmap_changed_l1), int32 [k, 3]."""
        k = int(lib().lo_voxelmap_changed_l1(self._h, None, 0))
        out = np.zeros((max(k, 1), 3), np.int32)
        got = lib().lo_voxelmap_changed_l1(self._h, out.ctypes.data_as(C.POINTER(C.c_int32)), k)
        return out[:min(got, k)]

    def surfel_at(self, p):
        """GetSurfelAtPoint (VoxelMap.cpp:368-386): (normal, centroid) of p's L1 voxel surfel, or None."""
        q = np.ascontiguousarray(p, np.float32).reshape(3)
        n = np.zeros(3, np.float32)
        c = np.zeros(3, np.float32)
        return (n, c) if lib().lo_voxelmap_surfel_at(self._h, _f(q), _f(n), _f(c)) else None

    def l0_cloud(self) -> np.ndarray:
        """VoxelMap::GetPointCloud (VoxelMap.cpp:388-403)."""
        m = self.l0_count()
        out = np.zeros((max(m, 1), 3), np.float32)
        got = lib().lo_voxelmap_get_l0(self._h, _f(out), m)
        return out[:got]


class DeviceVoxelMap:
    """The same map kept on the GPU next to an ICP context (``lo_devmap_*``, csrc/lo_devmap.hip): updates are kernel
    launches on the context's stream that also patch its surfel table; the containers equal :class:`VoxelMap`'s bit
    for bit.  ``icp`` is an IterativeClosestPointOptimizer in surfel mode; close this map before it."""

    def __init__(self, icp, voxel_size: float = 0.5, hierarchy_factor: int = 3, planarity_threshold: float = 0.1,
                 max_l0: int = 1 << 20, max_points: int = 1 << 18):
        self._L = lib()
        err = C.c_int(0)
        self._h = self._L.lo_devmap_create(icp.ctx, float(voxel_size), int(hierarchy_factor),
                                           float(planarity_threshold), int(max_l0), int(max_points), C.byref(err))
        if not self._h:
            raise RuntimeError(f"lo_devmap_create failed ({err.value})")
        self.icp = icp

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            self._h = None
            self._L.lo_devmap_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc < 0:
            raise RuntimeError(f"devmap error {rc}: {self._L.lo_devmap_last_error(self._h).decode()}")
        return rc

    def update(self, world_points, sensor_position, max_distance: float, is_keyframe: bool = True):
        """UpdateVoxelMap: world_points a host array or a CUDA tensor (float32 [n, 3], read by the kernels)."""
        s = np.ascontiguousarray(sensor_position, dtype=np.float64).reshape(3)
        sp = s.ctypes.data_as(C.POINTER(C.c_double))
        if hasattr(world_points, "is_cuda") and world_points.is_cuda:
            t = world_points.contiguous()
            self._keep = t
            self._check(self._L.lo_devmap_update(self._h, C.c_void_p(t.data_ptr()), t.shape[0], 1, sp,
                                                 float(max_distance), int(is_keyframe)))
        else:
            p = np.ascontiguousarray(world_points, dtype=np.float32).reshape(-1, 3)
            self._check(self._L.lo_devmap_update(self._h, p.ctypes.data_as(C.c_void_p), len(p), 0, sp,
                                                 float(max_distance), int(is_keyframe)))

    def apply_transform(self, T):
        t = np.ascontiguousarray(np.asarray(T, np.float32)[:3, :] if np.asarray(T).ndim == 2 else
                                 np.asarray(T, np.float32).reshape(12)).reshape(12)
        self._check(self._L.lo_devmap_apply_transform(self._h, _f(t)))

    def status(self) -> int:
        """lo_devmap_status: 0, or LO_ERR_CAPACITY when an update overflowed a capacity / met a key beyond +-2^20."""
        return int(self._L.lo_devmap_status(self._h))

    def counts(self):
        """(L0 voxels, L1 voxels, surfels); raises on an overflow / key error bit."""
        out = (C.c_size_t * 4)()
        self._check(self._L.lo_devmap_counts(self._h, out))
        return int(out[0]), int(out[1]), int(out[2])

    def l0(self):
        """(keys int32 [n,3], centroids [n,3], point counts [n]) in L0 order."""
        n = self.counts()[0]
        k = np.zeros((max(n, 1), 3), np.int32)
        c = np.zeros((max(n, 1), 3), np.float32)
        pc = np.zeros(max(n, 1), np.int32)
        got = self._L.lo_devmap_get_l0(self._h, k.ctypes.data_as(C.POINTER(C.c_int32)), _f(c),
                                       pc.ctypes.data_as(C.POINTER(C.c_int32)), n)
        return k[:got], c[:got], pc[:got]

    def l1(self):
        """dict of L1 arrays in L1 order: keys, has_surfel, normals, centroids, planarity, child_counts, children."""
        n = self.counts()[1]
        m = max(n, 1)
        d = dict(keys=np.zeros((m, 3), np.int32), has_surfel=np.zeros(m, np.uint8), normals=np.zeros((m, 3), np.float32),
                 centroids=np.zeros((m, 3), np.float32), planarity=np.zeros(m, np.float32),
                 child_counts=np.zeros(m, np.int32), children=np.zeros((m, 27, 3), np.int32))
        ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))  # noqa: E731
        got = self._L.lo_devmap_get_l1(self._h, ip(d["keys"]), d["has_surfel"].ctypes.data_as(C.POINTER(C.c_uint8)),
                                       _f(d["normals"]), _f(d["centroids"]), _f(d["planarity"]), ip(d["child_counts"]),
                                       ip(d["children"]), n)
        return {k: v[:got] for k, v in d.items()}

    def surfels(self):
        """(keys, normals, centroids, planarity) of the voxels with a surfel, L1 order (VoxelMap.surfels' form)."""
        d = self.l1()
        h = d["has_surfel"].astype(bool)
        return d["keys"][h], d["normals"][h], d["centroids"][h], d["planarity"][h]


def voxel_filter(points, voxel_size: float, stride: int = 1) -> np.ndarray:
    """FastVoxelFilter::filter (VoxelMap.h:73-104): stride + Morton-keyed voxel centroids, first-occurrence order."""
    p = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
    out = np.zeros_like(p)
    n = lib().lo_voxel_filter(_f(p), len(p), float(voxel_size), int(stride), _f(out))
    return out[:n].copy()
