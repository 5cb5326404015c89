"""CPU ORACLE for the ICP hot path — TEST INFRASTRUCTURE ONLY.

ctypes bindings to ``oracle/liblo_oracle.so`` (built from ``oracle/src/lo_oracle.cpp`` by
``oracle/Makefile``).  Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this package; the product (``lidar_odometry_amd``) never does.

Parity status: PKO pinned against reference golden vectors (tests/golden/pko_golden.jsonl);
Eigen-dependent parts are parity-unpinned against reference binaries (see lo_oracle.cpp header).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liblo_oracle.so")


class PkoCfg(C.Structure):
    _fields_ = [("min_scale_factor", C.c_double), ("max_scale_factor", C.c_double),
                ("num_alpha_segments", C.c_int), ("truncated_threshold", C.c_double),
                ("gmm_components", C.c_int), ("gmm_sample_size", C.c_int), ("kernel", C.c_int)]


class IcpCfg(C.Structure):
    _fields_ = [("max_iterations", C.c_int), ("translation_tolerance", C.c_double),
                ("rotation_tolerance", C.c_double), ("max_correspondence_distance", C.c_double),
                ("min_correspondence_points", C.c_int), ("use_robust_loss", C.c_int),
                ("robust_loss_delta", C.c_double), ("use_pko", C.c_int), ("loss_cauchy", C.c_int),
                ("pko", PkoCfg)]


class IterLog(C.Structure):
    _fields_ = [("pose", C.c_float * 12), ("n_corr", C.c_int), ("scale", C.c_double),
                ("alpha", C.c_double), ("cost", C.c_float), ("H", C.c_float * 21),
                ("g", C.c_float * 6), ("delta", C.c_float * 6)]


# pko_kernel_type -> PkoCfg.kernel (AdaptiveMEstimator.cpp:128-156: any other name is Cauchy)
PKO_KERNELS = {"huber": 0, "cauchy": 1, "tukey": 2, "welsch": 3, "gemanMcClure": 4, "pseudoHuber": 5}


def pko_kernel_id(name: str) -> int:
    return PKO_KERNELS.get(name, 1)


def kitti_pko_cfg() -> PkoCfg:
    """config/kitti.yaml:41-51 robust_estimation block (same values in mid360.yaml)."""
    return PkoCfg(0.1, 10.0, 100, 10.0, 3, 100, 0)


def kitti_icp_cfg(max_iterations: int = 4) -> IcpCfg:
    """ICPConfig as wired by Estimator.cpp:62-70 from config/kitti.yaml:34-38."""
    return IcpCfg(max_iterations, 0.005, 0.005, 1.0, 10, 1, 0.1, 1, 0, kitti_pko_cfg())


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"oracle library missing: {_LIB_PATH} (run `make -C oracle`)")
        L = C.CDLL(_LIB_PATH)
        dp, fp, ip, u8p, vp = (C.POINTER(C.c_double), C.POINTER(C.c_float), C.POINTER(C.c_int),
                               C.POINTER(C.c_uint8), C.c_void_p)
        L.or_pko_scale_factor.restype = C.c_double
        L.or_pko_scale_factor.argtypes = [C.POINTER(PkoCfg), dp, C.c_int, dp]
        L.or_shuffle_prefix.argtypes = [C.c_int, C.c_int, ip]
        L.or_kmeans_seed_draws.argtypes = [C.c_int, C.c_int, ip]
        L.or_pko_tables.argtypes = [C.POINTER(PkoCfg), dp, dp]
        L.or_se3_compose.argtypes = [fp, fp, fp]
        L.or_se3_inverse.argtypes = [fp, fp]
        L.or_keyframe_metrics.argtypes = [fp, fp, dp]
        L.or_so3_exp.argtypes = [fp, fp]
        L.or_so3_normalize.argtypes = [fp, fp]
        L.or_jacobi_svd3.argtypes = [fp, fp, fp, fp]
        L.or_jacobi_svd3.restype = C.c_int
        L.or_ldlt6_solve.argtypes = [fp, fp, fp]
        L.or_map_create.restype = vp
        L.or_map_create.argtypes = [C.c_float, C.c_int, C.c_float, C.c_int]
        L.or_map_destroy.argtypes = [vp]
        L.or_map_update.argtypes = [vp, fp, C.c_int, dp, C.c_double, C.c_int]
        L.or_map_apply_transform.argtypes = [vp, fp]
        for f in ("or_map_l0_count", "or_map_l1_count", "or_map_surfel_count"):
            getattr(L, f).argtypes = [vp]
            getattr(L, f).restype = C.c_int
        L.or_map_get_surfels.argtypes = [vp, C.POINTER(C.c_int32), fp, fp, fp, C.c_int]
        L.or_map_get_surfels.restype = C.c_int
        L.or_map_get_l0.argtypes = [vp, fp, C.c_int]
        L.or_map_get_l0.restype = C.c_int
        L.or_map_lookup.argtypes = [vp, fp, fp, fp]
        L.or_map_lookup.restype = C.c_int
        L.or_voxel_filter.argtypes = [fp, C.c_int, C.c_float, C.c_int, fp]
        L.or_voxel_filter.restype = C.c_int
        L.or_transform_points.argtypes = [fp, C.c_int, fp, fp]
        L.or_find_correspondences.argtypes = [vp, fp, C.c_int, fp, C.c_double, u8p, dp]
        L.or_find_correspondences.restype = C.c_int
        L.or_find_correspondences_kdtree.argtypes = [vp, fp, C.c_int, fp, C.c_double, u8p, dp, fp, fp]
        L.or_find_correspondences_kdtree.restype = C.c_int
        L.or_map_trace.argtypes = [vp, C.c_int]
        L.or_map_trace.restype = None
        L.or_map_trace_get.argtypes = [vp, ip, C.c_size_t]
        L.or_map_trace_get.restype = C.c_size_t
        L.or_map_orders.argtypes = [vp, ip, ip, ip, ip, C.c_size_t]
        L.or_map_orders.restype = C.c_size_t
        L.or_kdtree_knn5.argtypes = [fp, C.c_int, fp, C.c_int, C.c_int, ip, fp, ip]
        L.or_kdtree_knn5.restype = None
        L.or_set_kdtree_search.argtypes = [C.c_int]
        L.or_set_kdtree_search.restype = None
        L.or_icp_optimize.argtypes = [vp, fp, C.c_int, fp, fp, C.POINTER(IcpCfg), C.c_int,
                                      C.POINTER(IterLog), ip]
        L.or_icp_optimize.restype = C.c_int
        L.or_icp_optimize_loop.argtypes = [fp, C.c_int, fp, fp, C.c_int, fp, C.POINTER(IcpCfg), fp, fp,
                                           C.POINTER(IterLog), C.c_int, ip, ip]
        L.or_icp_optimize_loop.restype = C.c_int
        L.or_build_normal_equations.argtypes = [vp, fp, C.c_int, fp, C.POINTER(IcpCfg), C.c_double,
                                                C.c_double, fp, fp, fp]
        L.or_build_normal_equations.restype = C.c_int
        _lib = L
    return _lib


def _f32(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a, a.ctypes.data_as(C.POINTER(C.c_float))


def _f64(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(C.POINTER(C.c_double))


# ---------------------------------------------------------------- PKO
def pko_scale_factor(residuals, cfg: PkoCfg | None = None):
    """Returns (alpha, gmm dict) — AdaptiveMEstimator::calculate_scale_factor."""
    cfg = cfg or kitti_pko_cfg()
    r, rp = _f64(residuals)
    K = cfg.gmm_components
    gmm = np.zeros(3 * K, dtype=np.float64)
    a = lib().or_pko_scale_factor(C.byref(cfg), rp, len(r), gmm.ctypes.data_as(C.POINTER(C.c_double)))
    return a, {"w": gmm[:K].copy(), "mu": gmm[K:2 * K].copy(), "var": gmm[2 * K:].copy()}


def shuffle_prefix(n: int, k: int) -> np.ndarray:
    out = np.zeros(max(k, 1), dtype=np.int32)
    lib().or_shuffle_prefix(n, k, out.ctypes.data_as(C.POINTER(C.c_int)))
    return out[:min(k, n)]


def kmeans_seed_draws(m: int, count: int = 2) -> np.ndarray:
    out = np.zeros(count, dtype=np.int32)
    lib().or_kmeans_seed_draws(m, count, out.ctypes.data_as(C.POINTER(C.c_int)))
    return out


def pko_tables(cfg: PkoCfg | None = None):
    cfg = cfg or kitti_pko_cfg()
    a = np.zeros(cfg.num_alpha_segments + 1)
    z = np.zeros(cfg.num_alpha_segments + 1)
    lib().or_pko_tables(C.byref(cfg), a.ctypes.data_as(C.POINTER(C.c_double)), z.ctypes.data_as(C.POINTER(C.c_double)))
    return a, z


# ---------------------------------------------------------------- math
def se3_inverse(A):
    a, ap = _f32(A)
    o = np.zeros(12, np.float32)
    lib().or_se3_inverse(ap, o.ctypes.data_as(C.POINTER(C.c_float)))
    return o


def keyframe_metrics(kf, pose):
    """(|t - t_kf|, |Log(R_kf^-1 R)|) as Estimator::should_create_keyframe computes them."""
    a, ap = _f32(kf)
    b, bp = _f32(pose)
    o = np.zeros(2, np.float64)
    lib().or_keyframe_metrics(ap, bp, o.ctypes.data_as(C.POINTER(C.c_double)))
    return float(o[0]), float(o[1])


def odometry(raw_scans, stride=8, voxel=0.5, map_voxel=0.5, max_range=100.0, kf_dist=1.0, kf_rot=0.3, initial=None):
    """Estimator::process_frame without loop closure / PGO (Estimator.cpp:115-233), on the oracle primitives.
    Returns (poses (n, 12) float32, keyframe flags)."""
    I = np.eye(3, 4, dtype=np.float32).reshape(12)
    P0 = I if initial is None else np.ascontiguousarray(np.asarray(initial, np.float32)[:3, :4].reshape(12))
    m = VoxelMap(map_voxel, 3, 0.1, True)
    poses, kfs = [], []
    prev = vel = last_kf = I
    n_kf = 0
    for k, raw in enumerate(raw_scans):
        pts = voxel_filter(raw, voxel, stride)
        kf = False
        if k == 0:
            pose = P0
            kf = len(pts) > 0
        elif n_kf == 0:
            # empty first frame: no keyframe was made, so every later frame returns early (Estimator.cpp:140-144)
            poses.append(np.asarray(prev, np.float32).reshape(12))
            kfs.append(False)
            continue
        else:
            guess = se3_compose(prev, vel)
            g_in = guess.copy().reshape(3, 4)
            g_in[:, :3] = so3_normalize(g_in[:, :3].reshape(9)).reshape(3, 3)
            ok, T, _, _ = icp_optimize(m, pts, g_in.reshape(12))
            if ok:
                pose = np.asarray(T, np.float32).reshape(3, 4).copy()
                pose[:, :3] = so3_normalize(pose[:, :3].reshape(9)).reshape(3, 3)
                pose = pose.reshape(12)
            else:
                pose = guess
            vel = se3_compose(se3_inverse(prev), pose)
            d, a = keyframe_metrics(last_kf, pose)
            kf = d > kf_dist or a > kf_rot
        prev = pose
        if kf:
            n_kf += 1
            w = transform_points(pts, pose)
            m.update(w, np.asarray(pose, np.float32).reshape(3, 4)[:, 3].astype(np.float64), 1.2 * max_range, True)
            last_kf = pose
        poses.append(np.asarray(pose, np.float32).reshape(12))
        kfs.append(kf)
    return np.stack(poses), kfs


def se3_compose(A, B):
    a, ap = _f32(A)
    b, bp = _f32(B)
    o = np.zeros(12, np.float32)
    lib().or_se3_compose(ap, bp, o.ctypes.data_as(C.POINTER(C.c_float)))
    return o


def so3_exp(w):
    a, ap = _f32(w)
    o = np.zeros(9, np.float32)
    lib().or_so3_exp(ap, o.ctypes.data_as(C.POINTER(C.c_float)))
    return o.reshape(3, 3)


def so3_normalize(R):
    a, ap = _f32(np.asarray(R).reshape(9))
    o = np.zeros(9, np.float32)
    lib().or_so3_normalize(ap, o.ctypes.data_as(C.POINTER(C.c_float)))
    return o.reshape(3, 3)


def jacobi_svd3(A):
    a, ap = _f32(np.asarray(A).reshape(9))
    U = np.zeros(9, np.float32); S = np.zeros(3, np.float32); V = np.zeros(9, np.float32)
    rc = lib().or_jacobi_svd3(ap, U.ctypes.data_as(C.POINTER(C.c_float)), S.ctypes.data_as(C.POINTER(C.c_float)),
                              V.ctypes.data_as(C.POINTER(C.c_float)))
    return rc, U.reshape(3, 3), S, V.reshape(3, 3)


def ldlt6_solve(H, b):
    h, hp = _f32(np.asarray(H).reshape(36))
    bb, bp = _f32(b)
    x = np.zeros(6, np.float32)
    lib().or_ldlt6_solve(hp, bp, x.ctypes.data_as(C.POINTER(C.c_float)))
    return x


def transform_points(pts, T):
    p, pp = _f32(pts)
    t, tp = _f32(np.asarray(T).reshape(12))
    o = np.zeros_like(p)
    lib().or_transform_points(pp, len(p), tp, o.ctypes.data_as(C.POINTER(C.c_float)))
    return o


def voxel_filter(pts, voxel_size: float, stride: int):
    p, pp = _f32(pts)
    o = np.zeros_like(p)
    n = lib().or_voxel_filter(pp, len(p), voxel_size, stride, o.ctypes.data_as(C.POINTER(C.c_float)))
    return o[:n].copy()


# ---------------------------------------------------------------- map
class VoxelMap:
    """Restatement of map::VoxelMap (VoxelMap.cpp)."""

    def __init__(self, voxel_size=0.5, hierarchy_factor=3, planarity_threshold=0.1, compute_surfels=True):
        self.h = lib().or_map_create(voxel_size, hierarchy_factor, planarity_threshold, int(compute_surfels))

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_map_destroy(self.h)
            self.h = None

    def update(self, world_pts, sensor_pos, max_distance, is_keyframe=True):
        p, pp = _f32(world_pts)
        s, sp = _f64(sensor_pos)
        lib().or_map_update(self.h, pp, len(p), sp, float(max_distance), int(is_keyframe))

    def apply_transform(self, T):
        t, tp = _f32(np.asarray(T).reshape(12))
        lib().or_map_apply_transform(self.h, tp)

    def enable_trace(self, on=True):
        """Record the container-operation trace (insert / erase / clear on L0, L1, children; see lo_oracle.cpp)."""
        lib().or_map_trace(self.h, int(bool(on)))

    def trace(self):
        n = lib().or_map_trace_get(self.h, None, 0)
        out = np.zeros(n, np.int32)
        if n:
            lib().or_map_trace_get(self.h, out.ctypes.data_as(C.POINTER(C.c_int)), n)
        return out.reshape(-1, 7)

    def orders(self):
        """Iteration orders: (L0 keys (n0, 3), L1 keys (n1, 3), children per L1 (n1,), children keys (nc, 3))."""
        ip = C.POINTER(C.c_int)
        nc = lib().or_map_orders(self.h, None, None, None, None, 0)
        l0 = np.zeros((self.l0_count(), 3), np.int32)
        l1 = np.zeros((self.l1_count(), 3), np.int32)
        cnt = np.zeros(self.l1_count(), np.int32)
        ch = np.zeros((max(nc, 1), 3), np.int32)
        lib().or_map_orders(self.h, l0.ctypes.data_as(ip), l1.ctypes.data_as(ip), cnt.ctypes.data_as(ip),
                            ch.ctypes.data_as(ip), nc)
        return l0, l1, cnt, ch[:nc]

    def l0_count(self):
        return lib().or_map_l0_count(self.h)

    def l1_count(self):
        return lib().or_map_l1_count(self.h)

    def surfel_count(self):
        return lib().or_map_surfel_count(self.h)

    def surfels(self):
        m = self.surfel_count()
        keys = np.zeros((max(m, 1), 3), np.int32)
        nrm = np.zeros((max(m, 1), 3), np.float32)
        cen = np.zeros((max(m, 1), 3), np.float32)
        pl = np.zeros(max(m, 1), np.float32)
        k = lib().or_map_get_surfels(self.h, keys.ctypes.data_as(C.POINTER(C.c_int32)),
                                     nrm.ctypes.data_as(C.POINTER(C.c_float)), cen.ctypes.data_as(C.POINTER(C.c_float)),
                                     pl.ctypes.data_as(C.POINTER(C.c_float)), m)
        return keys[:k], nrm[:k], cen[:k], pl[:k]

    def l0_cloud(self):
        m = self.l0_count()
        out = np.zeros((max(m, 1), 3), np.float32)
        k = lib().or_map_get_l0(self.h, out.ctypes.data_as(C.POINTER(C.c_float)), m)
        return out[:k]

    def lookup(self, p):
        pp = np.ascontiguousarray(p, np.float32)
        n = np.zeros(3, np.float32); c = np.zeros(3, np.float32)
        ok = lib().or_map_lookup(self.h, pp.ctypes.data_as(C.POINTER(C.c_float)), n.ctypes.data_as(C.POINTER(C.c_float)),
                                 c.ctypes.data_as(C.POINTER(C.c_float)))
        return bool(ok), n, c


# ---------------------------------------------------------------- ICP
def kdtree_knn5(cloud, queries, use_tree=True):
    """util::KdTree::nearestKSearch(q, 5) (PointCloudUtils.h:398-423) on the restated nanoflann tree.
    Returns (idx (nq, 5) int32, dist (nq, 5) float32, found (nq,) int32); idx -1 / dist inf past `found`."""
    c, cp = _f32(np.asarray(cloud, np.float32).reshape(-1, 3))
    q, qp = _f32(np.asarray(queries, np.float32).reshape(-1, 3))
    nq = len(q)
    idx = np.full((nq, 5), -1, np.int32)
    dist = np.full((nq, 5), np.inf, np.float32)
    found = np.zeros(nq, np.int32)
    ip = C.POINTER(C.c_int)
    fp = C.POINTER(C.c_float)
    lib().or_kdtree_knn5(cp, len(c), qp, nq, int(bool(use_tree)),
                         idx.ctypes.data_as(ip), dist.ctypes.data_as(fp), found.ctypes.data_as(ip))
    return idx, dist, found


def set_kdtree_search(use_tree: bool):
    """KDTree-variant neighbour search: kd-tree (default) or the index-ordered brute force (same results)."""
    lib().or_set_kdtree_search(int(bool(use_tree)))


def find_correspondences(vmap: VoxelMap, pts, T, max_corr=1.0, kdtree=False):
    p, pp = _f32(pts)
    t, tp = _f32(np.asarray(T).reshape(12))
    valid = np.zeros(len(p), np.uint8)
    res = np.zeros(len(p), np.float64)
    if kdtree:
        n = lib().or_find_correspondences_kdtree(vmap.h, pp, len(p), tp, max_corr, valid.ctypes.data_as(C.POINTER(C.c_uint8)),
                                                 res.ctypes.data_as(C.POINTER(C.c_double)), None, None)
    else:
        n = lib().or_find_correspondences(vmap.h, pp, len(p), tp, max_corr, valid.ctypes.data_as(C.POINTER(C.c_uint8)),
                                          res.ctypes.data_as(C.POINTER(C.c_double)))
    return n, valid.astype(bool), res


def icp_optimize(vmap: VoxelMap, pts, T_init, cfg: IcpCfg | None = None, kdtree=False):
    """Returns (ok, T_out[12], iterations, logs list of dicts)."""
    cfg = cfg or kitti_icp_cfg()
    p, pp = _f32(pts)
    t, tp = _f32(np.asarray(T_init).reshape(12))
    To = np.zeros(12, np.float32)
    logs = (IterLog * max(cfg.max_iterations, 1))()
    iters = C.c_int(0)
    ok = lib().or_icp_optimize(vmap.h, pp, len(p), tp, To.ctypes.data_as(C.POINTER(C.c_float)), C.byref(cfg),
                               int(kdtree), logs, C.byref(iters))
    out = []
    for i in range(iters.value):
        L = logs[i]
        out.append({"pose": np.array(L.pose[:], np.float32), "n_corr": L.n_corr, "scale": L.scale, "alpha": L.alpha,
                    "cost": L.cost, "H": np.array(L.H[:], np.float32), "g": np.array(L.g[:], np.float32),
                    "delta": np.array(L.delta[:], np.float32)})
    return bool(ok), To, iters.value, out


def _logs_list(logs, n):
    out = []
    for i in range(n):
        L = logs[i]
        out.append({"pose": np.array(L.pose[:], np.float32), "n_corr": L.n_corr, "scale": L.scale, "alpha": L.alpha,
                    "cost": L.cost, "H": np.array(L.H[:], np.float32), "g": np.array(L.g[:], np.float32),
                    "delta": np.array(L.delta[:], np.float32)})
    return out


def icp_optimize_loop(curr, T_curr, matched, T_matched, cfg: IcpCfg | None = None, max_logs=100):
    """optimize_loop (IterativeClosestPointOptimizer.cpp:40-251).  Returns (ok, converged, T_rel[12] or None,
    inlier_ratio or None, iterations, logs); T_rel / inlier_ratio exist only when the iteration converged."""
    cfg = cfg or kitti_icp_cfg()
    c, cp = _f32(np.asarray(curr).reshape(-1, 3))
    m, mp = _f32(np.asarray(matched).reshape(-1, 3))
    def p12(T):
        a = np.asarray(T, np.float32)
        return a.reshape(12) if a.size == 12 else a[:3, :4].reshape(12)
    tc, tcp = _f32(p12(T_curr))
    tm, tmp = _f32(p12(T_matched))
    Tr = np.zeros(12, np.float32)
    inl = C.c_float(0.0)
    logs = (IterLog * max_logs)()
    iters, conv = C.c_int(0), C.c_int(0)
    ok = lib().or_icp_optimize_loop(cp, len(c), tcp, mp, len(m), tmp, C.byref(cfg), Tr.ctypes.data_as(C.POINTER(C.c_float)),
                                    C.byref(inl), logs, max_logs, C.byref(iters), C.byref(conv))
    cv = bool(conv.value)
    return bool(ok), cv, (Tr if cv else None), (inl.value if cv else None), iters.value, _logs_list(logs, min(iters.value, max_logs))


def build_normal_equations(vmap: VoxelMap, pts, T, scale, delta, cfg: IcpCfg | None = None):
    cfg = cfg or kitti_icp_cfg()
    p, pp = _f32(pts)
    t, tp = _f32(np.asarray(T).reshape(12))
    H = np.zeros(36, np.float32); g = np.zeros(6, np.float32); cost = C.c_float(0)
    n = lib().or_build_normal_equations(vmap.h, pp, len(p), tp, C.byref(cfg), float(scale), float(delta),
                                        H.ctypes.data_as(C.POINTER(C.c_float)), g.ctypes.data_as(C.POINTER(C.c_float)),
                                        C.byref(cost))
    return n, H.reshape(6, 6), g, cost.value
