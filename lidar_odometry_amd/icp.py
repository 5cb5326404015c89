"""Host-side mirror of the reference's ICP interface over the HIP C ABI.

``IterativeClosestPointOptimizer`` keeps the reference's names, argument meaning and error behaviour
(src/optimization/IterativeClosestPointOptimizer.h:148-215):

* ``optimize(voxel_map, points, initial_transform)`` -> ``(success, optimized_transform)``; on failure
  (fewer than ``min_correspondence_points`` correspondences in some iteration) it returns ``False`` and the
  initial transform, exactly like ``optimize`` (:298-302 with :266).
* ``get_last_stats()`` mirrors ``OptimizationStats`` (:192-199) plus per-iteration logs.

Every call runs on the GPU through ``liblo_icp.so``; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import LO_ERR_CAPACITY, LoBatchRec, LoConfig, LoIterLog, LoStats, lib


@dataclass
class ICPConfig:
    """ICPConfig (IterativeClosestPointOptimizer.h:55-76) as Estimator.cpp:62-70 wires it from kitti.yaml."""
    max_iterations: int = 4
    translation_tolerance: float = 0.005
    rotation_tolerance: float = 0.005
    max_correspondence_distance: float = 1.0
    min_correspondence_points: int = 10
    use_robust_loss: bool = True
    robust_loss_delta: float = 0.1
    use_surfel_correspondence: bool = True


@dataclass
class AdaptiveMEstimatorConfig:
    """AdaptiveMEstimatorConfig (AdaptiveMEstimator.h:24-41) with config/kitti.yaml:41-51 values."""
    use_adaptive_m_estimator: bool = True
    loss_type: str = "huber"            # SystemConfig.loss_type is never parsed (ConfigUtils.h:65)
    min_scale_factor: float = 0.1
    max_scale_factor: float = 10.0
    num_alpha_segments: int = 100
    truncated_threshold: float = 10.0
    gmm_components: int = 3
    gmm_sample_size: int = 100
    pko_kernel_type: str = "huber"


@dataclass
class MapGeometry:
    voxel_size: float = 0.5              # map_voxel_size (kitti.yaml:19)
    hierarchy_factor: int = 3            # Estimator.cpp:79


def make_config(icp: ICPConfig, pko: AdaptiveMEstimatorConfig, geom: MapGeometry, max_points: int) -> LoConfig:
    c = LoConfig()
    lib().lo_config_default_kitti(C.byref(c))
    c.max_iterations = icp.max_iterations
    c.translation_tolerance = icp.translation_tolerance
    c.rotation_tolerance = icp.rotation_tolerance
    c.max_correspondence_distance = icp.max_correspondence_distance
    c.min_correspondence_points = icp.min_correspondence_points
    c.use_robust_loss = int(icp.use_robust_loss)
    c.robust_loss_delta = icp.robust_loss_delta
    c.loss_cauchy = int(pko.loss_type == "cauchy")
    c.use_adaptive_m_estimator = int(pko.use_adaptive_m_estimator)
    c.min_scale_factor = pko.min_scale_factor
    c.max_scale_factor = pko.max_scale_factor
    c.num_alpha_segments = pko.num_alpha_segments
    c.truncated_threshold = pko.truncated_threshold
    c.gmm_components = pko.gmm_components
    c.gmm_sample_size = pko.gmm_sample_size
    # every pko_kernel_type of AdaptiveMEstimator.cpp:128-156; an unknown name is Cauchy there, and here
    c.pko_kernel = lib().lo_pko_kernel_from_name(pko.pko_kernel_type.encode())
    c.voxel_size = geom.voxel_size
    c.hierarchy_factor = geom.hierarchy_factor
    c.use_surfel_correspondence = int(icp.use_surfel_correspondence)
    c.max_points = int(max_points)
    return c


def _fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _as_pts(points) -> np.ndarray:
    p = np.ascontiguousarray(points, dtype=np.float32)
    if p.ndim != 2 or p.shape[1] != 3:
        raise ValueError("points must be an (N, 3) float32 array (Point3D AoS)")
    return p


def _as_pose(T) -> np.ndarray:
    T = np.ascontiguousarray(np.asarray(T, dtype=np.float32))
    if T.shape == (4, 4):
        T = np.ascontiguousarray(T[:3, :])
    return np.ascontiguousarray(T.reshape(12))


def pose34(T12) -> np.ndarray:
    return np.asarray(T12, dtype=np.float32).reshape(3, 4)


@dataclass
class OptimizationStats:
    num_correspondences: int = 0
    num_iterations: int = 0
    initial_cost: float = 0.0
    final_cost: float = 0.0
    optimization_time_ms: float = 0.0
    converged: bool = False
    iterations: list = field(default_factory=list)


class IterativeClosestPointOptimizer:
    """GPU point-to-plane ICP with PKO robust weights (one HIP context = one device + stream)."""

    def __init__(self, config: ICPConfig | None = None, adaptive: AdaptiveMEstimatorConfig | None = None,
                 geometry: MapGeometry | None = None, device: int = 0, max_points: int = 1 << 17):
        self.config = config or ICPConfig()
        self.adaptive = adaptive or AdaptiveMEstimatorConfig()
        self.geometry = geometry or MapGeometry()
        self._cfg = make_config(self.config, self.adaptive, self.geometry, max_points)
        err = C.c_int(0)
        self._L = lib()
        self._ctx = self._L.lo_create(C.byref(self._cfg), device, C.byref(err))
        if not self._ctx:
            raise RuntimeError(f"lo_create failed (code {err.value}); is a HIP device present?")
        self._map_token = None
        self._last = OptimizationStats()

    # ------------------------------------------------------------------ lifetime
    def surfel_count(self) -> int:
        """Surfels in the device table (lo_map_surfel_count)."""
        return int(self._L.lo_map_surfel_count(self.ctx))

    def set_exact(self, enable: bool = True):
        """Arithmetic mode (lo_set_exact): True = reference-exact (sequential fp32 sums, sorted-order scale, fp32 LDLT /
        SVD SO3; bit-identical to the reference restatement) -- the DEFAULT of every context; False = the opt-in fast mode
        (fp64 tree sums; within 1e-7 per step but not parity-safe where a PKO alpha nearly ties)."""
        rc = self._L.lo_set_exact(self.ctx, int(bool(enable)))
        if rc != 0:
            raise RuntimeError(f"lo_set_exact failed ({rc})")

    def set_pipeline(self, enable: bool = True, main_iterations: int = 0):
        """Scan pipeline (default on): GN iterations >= main_iterations run on the context's tail stream and the context
        stream waits only for the scan's final result; results are identical either way (lo_set_pipeline)."""
        rc = self._L.lo_set_pipeline(self.ctx, int(bool(enable)), int(main_iterations))
        if rc != 0:
            raise RuntimeError(f"lo_set_pipeline failed ({rc})")

    def close(self):
        h = getattr(self, "_ctx", None)
        if h:
            self._ctx = None
            self._L.lo_destroy(h)

    def __del__(self):
        # at interpreter teardown module globals (lib, os) may already be None: the handle keeps its own
        # reference to the loaded library, and a destructor never raises
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc < 0:
            raise RuntimeError(f"liblo_icp error {rc}: {lib().lo_last_error(self._ctx).decode()}")
        return rc

    @property
    def ctx(self):
        return self._ctx

    # ------------------------------------------------------------------ map
    def set_surfels(self, keys, normals, centroids):
        """Upload the L1 surfels (VoxelMap nodes with has_surfel) as the device hash table."""
        k = np.ascontiguousarray(keys, dtype=np.int32).reshape(-1, 3)
        n = np.ascontiguousarray(normals, dtype=np.float32).reshape(-1, 3)
        c = np.ascontiguousarray(centroids, dtype=np.float32).reshape(-1, 3)
        if not (len(k) == len(n) == len(c)):
            raise ValueError("keys/normals/centroids length mismatch")
        self._check(lib().lo_map_set_surfels(self._ctx, k.ctypes.data_as(C.POINTER(C.c_int32)), _fptr(n), _fptr(c), len(k)))

    def sync_surfels(self, keys, normals, centroids) -> int:
        """The map's whole current surfel set after UpdateVoxelMap; only the difference to the last sync is patched into
        the device table (lo_map_sync_surfels).  Returns the records sent, -1 after a full upload."""
        k = np.ascontiguousarray(keys, dtype=np.int32).reshape(-1, 3)
        n = np.ascontiguousarray(normals, dtype=np.float32).reshape(-1, 3)
        c = np.ascontiguousarray(centroids, dtype=np.float32).reshape(-1, 3)
        if not (len(k) == len(n) == len(c)):
            raise ValueError("keys/normals/centroids length mismatch")
        patched = C.c_int(0)
        self._check(lib().lo_map_sync_surfels(self._ctx, k.ctypes.data_as(C.POINTER(C.c_int32)), _fptr(n), _fptr(c),
                                              len(k), C.byref(patched)))
        return int(patched.value)

    def sync_changed(self, voxel_map, changed_keys) -> int:
        """The keyed sync after UpdateVoxelMap (the adapter's sync_map(vm, changed)): only the L1 voxels the update
        changed (``VoxelMap.changed_l1()``; in the reference, the keys the INTEGRATION.md hook collects) are looked up
        with GetSurfelAtPoint at the key's voxel centre and patched in place (lo_map_patch_surfels): a surfel is
        upserted, a voxel without one erased.  The map must have been uploaded whole before (set_surfels /
        sync_surfels).  Returns the records sent."""
        keys = np.ascontiguousarray(changed_keys, np.int32).reshape(-1, 3)
        if len(keys) == 0:
            return 0
        n = np.zeros((len(keys), 3), np.float32)
        c = np.zeros((len(keys), 3), np.float32)
        pres = np.zeros(len(keys), np.uint8)
        # the adapter's per-key GetSurfelAtPoint loop, in one call on this library's host map
        lib().lo_voxelmap_surfels_at_keys(voxel_map.handle, keys.ctypes.data_as(C.POINTER(C.c_int32)), len(keys),
                                          _fptr(n), _fptr(c), pres.ctypes.data)
        rc = lib().lo_map_patch_surfels(self._ctx, keys.ctypes.data, n.ctypes.data, c.ctypes.data, pres.ctypes.data,
                                        len(keys))
        if rc == LO_ERR_CAPACITY:                 # tombstones: a whole upload rebuilds the table (as the adapter does)
            s = voxel_map.surfels()
            self.set_surfels(s[0], s[1], s[2])
            return -1
        self._check(rc)
        return len(keys)

    def update_config(self, config: ICPConfig, adaptive: AdaptiveMEstimatorConfig | None = None):
        """IterativeClosestPointOptimizer::update_config (IterativeClosestPointOptimizer.h:220): new parameters, same
        context -- the device map stays (lo_update_config).  adaptive: new PKO parameters too (the estimator's config)."""
        ad = adaptive or self.adaptive
        cfg = make_config(config, ad, self.geometry, self._cfg.max_points)
        self._check(self._L.lo_update_config(self.ctx, C.byref(cfg)))
        self.config = config
        self.adaptive = ad
        self._cfg = cfg

    def get_config(self) -> ICPConfig:
        return self.config

    def set_map_points(self, points):
        """KDTree variant: upload VoxelMap::GetPointCloud (L0 centroids, L0 order) -- RebuildKdTree's input."""
        p = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
        self._check(lib().lo_map_set_points(self._ctx, _fptr(p), len(p)))

    def _sync_map(self, voxel_map):
        if voxel_map is None:
            return
        token = (id(voxel_map), getattr(voxel_map, "revision", None))
        if token == self._map_token and token[1] is not None:
            return
        if self.config.use_surfel_correspondence:
            s = voxel_map.surfels()
            self.set_surfels(s[0], s[1], s[2])
        else:
            self.set_map_points(voxel_map.l0_cloud())
        self._map_token = token

    # ------------------------------------------------------------------ optimize
    def optimize(self, voxel_map, points, initial_transform):
        """IterativeClosestPointOptimizer::optimize -> (success, optimized_transform[3x4])."""
        self._sync_map(voxel_map)
        p = _as_pts(points)
        Ti = _as_pose(initial_transform)
        To = np.zeros(12, np.float32)
        logs = (LoIterLog * self._cfg.max_iterations)()
        st = LoStats()
        rc = self._check(lib().lo_icp_optimize(self._ctx, _fptr(p), len(p), _fptr(Ti), _fptr(To), logs, C.byref(st)))
        self._record(st, logs)
        return rc == _lib.LO_OK, pose34(To)

    def optimize_raw(self, voxel_map, raw_points, initial_transform, stride: int = 8, voxel_size: float = 0.5):
        """Estimator::preprocess_frame (FastVoxelFilter on the device) + optimize, no host round trip between them."""
        self._sync_map(voxel_map)
        p = _as_pts(raw_points)
        Ti = _as_pose(initial_transform)
        To = np.zeros(12, np.float32)
        logs = (LoIterLog * self._cfg.max_iterations)()
        st = LoStats()
        rc = self._check(lib().lo_icp_optimize_raw(self._ctx, _fptr(p), len(p), int(stride), float(voxel_size),
                                                   _fptr(Ti), _fptr(To), logs, C.byref(st)))
        self._record(st, logs)
        return rc == _lib.LO_OK, pose34(To)

    def optimize_loop(self, curr_points, curr_pose, matched_points, matched_pose):
        """IterativeClosestPointOptimizer::optimize_loop (IterativeClosestPointOptimizer.cpp:40-251) on the device:
        the two keyframes' feature clouds (local frames) and world poses.  Returns (success, T_rel, inlier_ratio);
        as the reference, T_rel (= curr_pose^-1 * optimized pose, 3x4) and inlier_ratio are None unless the
        iteration converged.  The context's own map is not touched."""
        c = _as_pts(curr_points)
        m = _as_pts(matched_points)
        Tc, Tm = _as_pose(curr_pose), _as_pose(matched_pose)
        Tr = np.zeros(12, np.float32)
        inl = C.c_float(0.0)
        logs = (LoIterLog * _lib.LO_MAX_ITERS)()
        st = LoStats()
        rc = self._check(lib().lo_icp_optimize_loop(self._ctx, _fptr(c), len(c), _fptr(Tc), _fptr(m), len(m), _fptr(Tm),
                                                    _fptr(Tr), C.byref(inl), logs, C.byref(st)))
        self._record(st, logs)
        conv = bool(st.converged)
        return rc == _lib.LO_OK, (pose34(Tr) if conv else None), (inl.value if conv else None)

    def filtered_points(self) -> np.ndarray:
        """Feature cloud of the last device-filtered scan (for the keyframe map update)."""
        n = self._check(lib().lo_filtered_points(self._ctx, None, 0))
        out = np.zeros((max(n, 1), 3), np.float32)
        self._check(lib().lo_filtered_points(self._ctx, _fptr(out), n))
        return out[:n]

    def voxel_filter(self, raw_points, voxel_size: float, stride: int = 1) -> np.ndarray:
        """FastVoxelFilter::filter on the device (parity entry; synchronous)."""
        p = _as_pts(raw_points)
        m = (len(p) + stride - 1) // stride
        out = np.zeros((max(m, 1), 3), np.float32)
        n = self._check(lib().lo_voxel_filter_gpu(self._ctx, _fptr(p), len(p), float(voxel_size), int(stride),
                                                  _fptr(out), max(m, 1)))
        return out[:n]

    def _record(self, st, logs):
        its = []
        for i in range(min(st.iterations, len(logs))):
            L = logs[i]
            its.append({"pose": np.array(L.pose[:], np.float32), "n_corr": L.n_corr, "scale": L.scale,
                        "alpha": L.alpha, "cost": L.cost, "H": np.array(L.H[:], np.float32),
                        "g": np.array(L.g[:], np.float32), "delta": np.array(L.delta[:], np.float32)})
        self._last = OptimizationStats(st.n_corr, st.iterations, st.initial_cost, st.final_cost, st.gpu_ms,
                                       bool(st.converged), its)

    def get_last_stats(self) -> OptimizationStats:
        return self._last

    # ------------------------------------------------------------------ single stages (parity harness)
    def find_correspondences(self, points, T):
        p = _as_pts(points)
        t = _as_pose(T)
        valid = np.zeros(len(p), np.uint8)
        res = np.zeros(len(p), np.float64)
        n = self._check(lib().lo_find_correspondences(self._ctx, _fptr(p), len(p), _fptr(t),
                                                      valid.ctypes.data_as(C.POINTER(C.c_uint8)),
                                                      res.ctypes.data_as(C.POINTER(C.c_double))))
        return n, valid.astype(bool), res

    def nearest_k_search(self, queries):
        """util::KdTree::nearestKSearch(q, 5) for world-frame queries over the map cloud (KDTree configuration):
        (idx (n, 5) int32, dist (n, 5) float32, found (n,) int32 = 5 or 0)."""
        q = _as_pts(queries)
        idx = np.full((len(q), 5), -1, np.int32)
        dist = np.full((len(q), 5), np.inf, np.float32)
        self._check(lib().lo_knn_search(self._ctx, _fptr(q), len(q), idx.ctypes.data_as(C.POINTER(C.c_int32)),
                                        dist.ctypes.data_as(C.POINTER(C.c_float))))
        return idx, dist, np.where(idx[:, 0] >= 0, 5, 0).astype(np.int32)

    def pko_scale_factor(self, residuals):
        r = np.ascontiguousarray(residuals, dtype=np.float64)
        K = self._cfg.gmm_components
        gmm = np.zeros(3 * K, np.float64)
        a = lib().lo_pko_scale_factor(self._ctx, r.ctypes.data_as(C.POINTER(C.c_double)), len(r),
                                      gmm.ctypes.data_as(C.POINTER(C.c_double)))
        if np.isnan(a):
            raise RuntimeError(f"lo_pko_scale_factor failed: {lib().lo_last_error(self._ctx).decode()}")
        return a, {"w": gmm[:K].copy(), "mu": gmm[K:2 * K].copy(), "var": gmm[2 * K:].copy()}

    def build_normal_equations(self, points, T, scale, delta):
        p = _as_pts(points)
        t = _as_pose(T)
        H = np.zeros(36, np.float64)
        g = np.zeros(6, np.float64)
        cost = C.c_double(0.0)
        n = self._check(lib().lo_build_normal_equations(self._ctx, _fptr(p), len(p), _fptr(t), float(scale),
                                                        float(delta), H.ctypes.data_as(C.POINTER(C.c_double)),
                                                        g.ctypes.data_as(C.POINTER(C.c_double)), C.byref(cost)))
        return n, H.reshape(6, 6), g, cost.value

    def pko_sample_indices(self, n):
        out = np.zeros(max(self._cfg.gmm_sample_size, 1), np.int32)
        k = self._check(lib().lo_pko_sample_indices(self._ctx, n, out.ctypes.data_as(C.POINTER(C.c_int32))))
        return out[:k]


@dataclass
class BatchResult:
    """One job of a batched optimize: the fields of lo_batch_rec."""
    success: bool
    pose: np.ndarray
    iterations: int
    n_corr: int
    initial_cost: float
    final_cost: float
    alpha: float


class BatchOptimizer:
    """Scan-parallel optimize on one GPU (lo_batch_*): B independent contexts -- B sequences, each with its own
    map and GN state -- run IterativeClosestPointOptimizer::optimize in lockstep, one launch per kernel per GN
    iteration for all of them.  Each job's result equals ``optimizers[j].optimize`` on the same input."""

    def __init__(self, optimizers):
        self.optimizers = list(optimizers)
        arr = (C.c_void_p * len(self.optimizers))(*[o.ctx for o in self.optimizers])
        err = C.c_int(0)
        self._L = lib()
        self._b = self._L.lo_batch_create(arr, len(self.optimizers), C.byref(err))
        if not self._b:
            raise RuntimeError(f"lo_batch_create failed (code {err.value})")
        self.last_gpu_ms = 0.0

    def close(self):
        h = getattr(self, "_b", None)
        if h:
            self._b = None
            self._L.lo_batch_destroy(h)

    def __del__(self):
        # at interpreter teardown module globals (lib, os) may already be None: the handle keeps its own
        # reference to the loaded library, and a destructor never raises
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return len(self.optimizers)

    def _check(self, rc):
        if rc < 0:
            raise RuntimeError(f"liblo_icp batch error {rc}: {lib().lo_batch_last_error(self._b).decode()}")
        return rc

    @staticmethod
    def _results(recs):
        out = []
        for r in recs:
            out.append(BatchResult(r.status == _lib.LO_OK, pose34(np.ctypeslib.as_array(r.pose).copy()),
                                   r.iterations, r.n_corr, r.initial_cost, r.final_cost, r.alpha))
        return out

    def optimize(self, voxel_maps, scans, initial_transforms):
        """Host scans in; returns one BatchResult per job.  voxel_maps (nullable entries) are synced per context."""
        B = len(self.optimizers)
        if voxel_maps is not None:
            for o, vm in zip(self.optimizers, voxel_maps):
                o._sync_map(vm)
        pts = [_as_pts(p) for p in scans]
        if len(pts) != B:
            raise ValueError(f"need {B} scans")
        T = np.ascontiguousarray(np.stack([_as_pose(t) for t in initial_transforms]), dtype=np.float32)
        ptrs = (C.c_void_p * B)(*[p.ctypes.data for p in pts])
        ns = (C.c_size_t * B)(*[len(p) for p in pts])
        recs = (LoBatchRec * B)()
        self._check(lib().lo_batch_optimize(self._b, ptrs, ns, _fptr(T), recs))
        return self._results(recs)

    def optimize_async(self, device_ptrs, counts, initial_transforms):
        """Device-resident scans (int device pointers, or 0 for the context's last uploaded scan)."""
        B = len(self.optimizers)
        self._T = np.ascontiguousarray(np.asarray(initial_transforms, dtype=np.float32).reshape(B, 12))
        ptrs = (C.c_void_p * B)(*[int(p) if p else None for p in device_ptrs])
        ns = (C.c_size_t * B)(*[int(n) for n in counts])
        self._check(lib().lo_batch_optimize_async(self._b, ptrs, ns, _fptr(self._T)))

    def result(self):
        B = len(self.optimizers)
        recs = (LoBatchRec * B)()
        ms = C.c_double(0.0)
        self._check(lib().lo_batch_result(self._b, recs, C.byref(ms)))
        self.last_gpu_ms = ms.value
        return self._results(recs)
