"""Per-iteration device-vs-oracle comparison of the loop-closure ICP (diagnostic, run on the GPU box)."""
import sys
import numpy as np

sys.path.insert(0, ".")
import oracle  # noqa: E402
from tests import _data  # noqa: E402
from lidar_odometry_amd import IterativeClosestPointOptimizer  # noqa: E402


def err(Ta, Tb):
    A = np.asarray(Ta, np.float64).reshape(3, 4)
    B = np.asarray(Tb, np.float64).reshape(3, 4)
    return float(np.linalg.norm(A[:, 3] - B[:, 3])), _data.rot_angle(A[:, :3], B[:, :3])


icp = IterativeClosestPointOptimizer(max_points=1 << 17)
for fa, fb, s in [(2, 6, 0), (4, 7, 3), (10, 14, 5), (20, 23, 9), (6, 9, 1), (12, 16, 2)]:
    cur, Tc, mat, Tm, _ = _data.loop_case(fa, fb, s)
    ok_o, conv_o, Tr_o, inl_o, it_o, logs_o = oracle.icp_optimize_loop(cur, Tc, mat, Tm)
    ok_g, Tr_g, inl_g = icp.optimize_loop(cur, Tc, mat, Tm)
    st = icp.get_last_stats()
    print(f"pair {fa}-{fb}: ok {ok_g}/{ok_o} iters {st.num_iterations}/{it_o} inl {inl_g}/{inl_o} gpu_ms {st.optimization_time_ms:.3f}")
    for k, (lo, lg) in enumerate(zip(logs_o, st.iterations)):
        et, er = err(lg["pose"], lo["pose"])
        dd = np.abs(np.asarray(lg["delta"], np.float64) - np.asarray(lo["delta"], np.float64)).max()
        print(f"  it {k}: n_corr {lg['n_corr']}/{lo['n_corr']} alpha {lg['alpha']:.6f}/{lo['alpha']:.6f} "
              f"scale {lg['scale']:.9f}/{lo['scale']:.9f} dt {et:.2e} dr {er:.2e} |ddelta| {dd:.2e} "
              f"|delta| {np.abs(lo['delta']).max():.2e}")
icp.close()
