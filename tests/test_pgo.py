"""Pose-graph optimisation (PGO half): lidar_odometry_amd.pgo.PoseGraphOptimizer (csrc/lo_pgo.cpp)
against the reference's PoseGraphOptimizer semantics (src/optimization/PoseGraphOptimizer.cpp:162-392).

Parity unpinned: the reference solves with Eigen::SimplicialLDLT and projects with Eigen::JacobiSVD, and Eigen is
absent here.  The restatement is checked (a) on pose graphs with a known optimum (exact measurements, drifted
initial estimates: the optimum is the ground truth), (b) against an independent dense numpy Gauss-Newton of the same
equations (GTSAM [rot, trans] order, error log(measured^-1 T_from^-1 T_to), J_from = -Ad(hx^-1), J_to = I,
T <- T Exp(dx), SVD re-projection), iteration for iteration, and (c) for the API's bookkeeping rules.
Host code only: no GPU.
"""
import numpy as np
import pytest

from lidar_odometry_amd.pgo import PoseGraphOptimizer

EPS = 1e-10


# ------------------------------------------------------------------ independent numpy restatement (fp64, dense)
def skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]], dtype=np.float64)


def so3_log(R):
    th = np.arccos(np.clip((np.trace(R) - 1) / 2, -1, 1))
    v = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    return v / 2 if th < EPS else v * (th / (2 * np.sin(th)))


def so3_exp(w):
    th = np.linalg.norm(w)
    if th < EPS:
        return np.eye(3) + skew(w)
    W = skew(w / th)
    return np.eye(3) + np.sin(th) * W + (1 - np.cos(th)) * W @ W


def se3_log(R, t):
    w = so3_log(R)
    th = np.linalg.norm(w)
    if th < EPS:
        return np.concatenate([w, t])
    W = skew(w / th)
    Wt = W @ t
    u = t - 0.5 * th * Wt + (1 - th / (2 * np.tan(0.5 * th))) * (W @ Wt)
    return np.concatenate([w, u])


def se3_exp(xi):
    w, u = xi[:3], xi[3:]
    R = so3_exp(w)
    th = np.linalg.norm(w)
    if th < EPS:
        return R, u.copy()
    W = skew(w)
    V = np.eye(3) + (1 - np.cos(th)) / th ** 2 * W + (th - np.sin(th)) / th ** 3 * W @ W
    return R, V @ u


def project(R):
    U, _, Vt = np.linalg.svd(R)
    M = U @ Vt
    if np.linalg.det(M) < 0:
        U[:, 2] *= -1
        M = U @ Vt
    return M


def sqrt_info(tn, rn):
    return np.array([1 / rn] * 3 + [1 / tn] * 3)


class NumpyPGO:
    def __init__(self):
        self.priors, self.betweens, self.poses, self.ids, self.index = [], [], {}, [], {}

    @staticmethod
    def _d(T):
        T = np.asarray(T, np.float32).astype(np.float64)
        return project(T[:3, :3]), T[:3, 3].copy()

    def first(self, kid, T):
        self.priors.append((0, self._d(T), sqrt_info(1e-4, 1e-4)))
        self.poses[kid] = self._d(T)
        self.ids.append(kid)
        self.index[kid] = 0

    def odom(self, prev, cur, T, rel, tn=0.1, rn=0.1):
        i = len(self.ids)
        if prev in self.index:
            self.betweens.append((self.index[prev], i, self._d(rel), sqrt_info(tn, rn)))
        else:
            self.priors.append((i, self._d(T), sqrt_info(0.5, 0.1)))
        self.poses[cur] = self._d(T)
        self.ids.append(cur)
        self.index[cur] = i

    def loop(self, a, b, rel, tn=0.05, rn=0.05):
        self.betweens.append((self.index[a], self.index[b], self._d(rel), sqrt_info(tn, rn)))
        return self.optimize()

    def optimize(self, max_it=10, thr=1e-6):
        n = len(self.ids)
        for it in range(max_it):
            H = np.zeros((6 * n, 6 * n))
            b = np.zeros(6 * n)
            for k, (Rm, tm), s in self.priors:
                R, t = self.poses[self.ids[k]]
                e = se3_log(Rm.T @ R, Rm.T @ (t - tm))
                H[6 * k:6 * k + 6, 6 * k:6 * k + 6] += np.diag(s * s)
                b[6 * k:6 * k + 6] -= s * (s * e)
            for f, t_, (Rm, tm), s in self.betweens:
                Ra, ta = self.poses[self.ids[f]]
                Rb, tb = self.poses[self.ids[t_]]
                Rhx, thx = Ra.T @ Rb, Ra.T @ (tb - ta)
                e = se3_log(Rm.T @ Rhx, Rm.T @ (thx - tm))
                Ri = Rhx.T
                ti = -Ri @ thx
                Ad = np.zeros((6, 6))
                Ad[:3, :3] = Ri
                Ad[3:, :3] = skew(ti) @ Ri
                Ad[3:, 3:] = Ri
                Jf = np.diag(s) @ -Ad
                Jt = np.diag(s)
                ew = s * e
                for (i, Ji), (j, Jj) in [((f, Jf), (f, Jf)), ((t_, Jt), (t_, Jt)), ((f, Jf), (t_, Jt)), ((t_, Jt), (f, Jf))]:
                    H[6 * i:6 * i + 6, 6 * j:6 * j + 6] += Ji.T @ Jj
                b[6 * f:6 * f + 6] -= Jf.T @ ew
                b[6 * t_:6 * t_ + 6] -= Jt.T @ ew
            dx = np.linalg.solve(H, b)
            for v in range(n):
                R, t = self.poses[self.ids[v]]
                dR, dt = se3_exp(dx[6 * v:6 * v + 6])
                self.poses[self.ids[v]] = (project(R @ dR), R @ dt + t)
            if np.linalg.norm(dx) < thr:
                return True, it + 1
        return False, max_it


# ------------------------------------------------------------------ synthetic graphs
def pose(R, t):
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return T


def trajectory(n, seed, loop_every=None):
    """A planar-ish drive (yaw turns, small pitch/roll), returning world poses (fp64 4x4)."""
    rng = np.random.default_rng(seed)
    Ts = [np.eye(4)]
    for k in range(1, n):
        w = np.array([rng.normal(0, 0.01), rng.normal(0, 0.01), rng.normal(0, 0.08)])
        step = pose(so3_exp(w), np.array([2.0 + rng.normal(0, 0.2), rng.normal(0, 0.05), rng.normal(0, 0.02)]))
        Ts.append(Ts[-1] @ step)
    return Ts


def rel(A, B):
    return np.linalg.inv(A) @ B


def noisy(T, rng, st, sr):
    return T @ pose(so3_exp(rng.normal(0, sr, 3)), rng.normal(0, st, 3))


def _err(A, B):
    A, B = np.asarray(A, np.float64), np.asarray(B, np.float64)
    dR = A[:3, :3].T @ B[:3, :3]
    return float(np.linalg.norm(A[:3, 3] - B[:3, 3])), float(np.linalg.norm(so3_log(dR)))


# ------------------------------------------------------------------ tests
def test_known_optimum_exact_measurements():
    """Odometry and loop measurements exact, initial estimates drifted: the optimum is the ground truth."""
    gt = trajectory(40, seed=3)
    rng = np.random.default_rng(5)
    p = PoseGraphOptimizer()
    try:
        est = [gt[0]]
        for k in range(1, len(gt)):
            est.append(noisy(est[-1] @ rel(gt[k - 1], gt[k]), rng, 0.05, 0.004))   # drifting dead reckoning
        assert p.add_first_keyframe(0, gt[0])
        for k in range(1, len(gt)):
            assert p.add_keyframe_with_odom(k - 1, k, est[k], rel(gt[k - 1], gt[k]))
        worst_before = max(_err(est[k], gt[k])[0] for k in range(len(gt)))
        assert worst_before > 0.5
        assert p.add_loop_and_optimize(39, 0, rel(gt[39], gt[0]))
        assert p.add_loop_and_optimize(30, 10, rel(gt[30], gt[10]))
        assert p.get_loop_closure_count() == 2
        got = p.get_all_optimized_poses()
        assert sorted(got) == list(range(40))
        for k in range(40):
            et, er = _err(got[k], gt[k])
            assert et < 2e-4 and er < 2e-6, (k, et, er)
    finally:
        p.close()


@pytest.mark.parametrize("seed", [1, 2])
def test_matches_dense_numpy_gauss_newton(seed):
    """Noisy odometry and loops (the optimum is a compromise): the same poses and iteration counts as a dense numpy
    Gauss-Newton of the same equations, after each loop closure."""
    gt = trajectory(60, seed=seed)
    rng = np.random.default_rng(seed + 100)
    p, q = PoseGraphOptimizer(), NumpyPGO()
    try:
        p.add_first_keyframe(0, gt[0])
        q.first(0, gt[0])
        est = gt[0]
        for k in range(1, len(gt)):
            z = noisy(rel(gt[k - 1], gt[k]), rng, 0.03, 0.003)
            est = est @ z
            p.add_keyframe_with_odom(k - 1, k, est, z)
            q.odom(k - 1, k, est.astype(np.float32), z.astype(np.float32))
        for a, b in [(59, 0), (45, 15), (50, 5)]:
            z = noisy(rel(gt[a], gt[b]), rng, 0.01, 0.001)
            assert p.add_loop_and_optimize(a, b, z)
            conv, its = q.loop(a, b, z.astype(np.float32))
            assert p.last_converged == conv and p.last_iterations == its
            got = p.get_all_optimized_poses()
            for k in range(len(gt)):
                R, t = q.poses[k]
                et, er = _err(got[k], pose(R, t))
                assert et < 5e-5 and er < 1e-6, (a, b, k, et, er)
    finally:
        p.close()


def test_bookkeeping_rules():
    """add_first_keyframe only on an empty graph; an existing keyframe is a no-op; an unknown previous keyframe gets
    a loose prior instead of an odometry factor; loops need both keyframes; clear() resets everything."""
    p = PoseGraphOptimizer()
    try:
        I = np.eye(4, dtype=np.float32)
        assert p.add_first_keyframe(7, I)
        assert not p.add_first_keyframe(8, I)
        T1 = pose(so3_exp(np.array([0, 0, 0.1])), [1.0, 0, 0]).astype(np.float32)
        assert p.add_keyframe_with_odom(7, 9, T1, T1)
        assert p.add_keyframe_with_odom(7, 9, I, I)          # exists: ignored
        ok, got = p.get_optimized_pose(9)
        assert ok and np.allclose(got, T1, atol=1e-6)
        T2 = pose(np.eye(3), [5.0, 5.0, 0]).astype(np.float32)
        assert p.add_keyframe_with_odom(100, 11, T2, I)       # unknown previous keyframe: loose prior at T2
        assert p.get_keyframe_count() == 3 and p.has_keyframe(11) and not p.has_keyframe(100)
        assert not p.add_loop_and_optimize(9, 12, I)          # unknown keyframe
        assert p.get_loop_closure_count() == 0
        assert p.add_loop_and_optimize(11, 7, rel(T2, I))      # consistent with the priors: nothing moves
        ok, got = p.get_optimized_pose(11)
        assert ok and np.allclose(got, T2, atol=1e-4)
        assert not p.get_optimized_pose(5)[0]
        assert list(p.get_all_optimized_poses()) == [7, 9, 11]
        p.clear()
        assert p.get_keyframe_count() == 0 and p.get_loop_closure_count() == 0 and not p.has_keyframe(7)
        assert p.add_first_keyframe(1, I)
    finally:
        p.close()


def test_long_chain_is_sparse_fast():
    """A 2000-keyframe chain with loop closures solves in well under a second per closure (envelope LDL^T: a chain
    keeps one block per row; the loop rows widen only their own envelope)."""
    gt = trajectory(2000, seed=9)
    rng = np.random.default_rng(9)
    p = PoseGraphOptimizer()
    try:
        p.add_first_keyframe(0, gt[0])
        est = gt[0]
        for k in range(1, len(gt)):
            z = noisy(rel(gt[k - 1], gt[k]), rng, 0.02, 0.002)
            est = est @ z
            p.add_keyframe_with_odom(k - 1, k, est, z)
        for a, b in [(1999, 0), (1500, 300)]:
            assert p.add_loop_and_optimize(a, b, rel(gt[a], gt[b]))
            assert p.last_converged
            assert p.last_ms < 1500.0, p.last_ms
        et, _ = _err(p.get_optimized_pose(1999)[1], gt[1999])
        e0, _ = _err(est, gt[1999])
        assert et < 0.1 * e0
    finally:
        p.close()
