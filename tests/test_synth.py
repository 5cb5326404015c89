"""Synthetic workload generators (CPU): the city-grid KITTI sequence behind bench.py's default map (12.8k surfels
after 660 frames, SURVEY.md §8d's 10^4-10^5 range; the bench line reports the count) is deterministic and drives on
its streets, with no building in the sensor's way."""
import numpy as np

from lidar_odometry_amd import synth


def test_city_sequence_deterministic_and_clear_of_buildings():
    a = synth.KittiCitySequence(n_frames=400)
    b = synth.KittiCitySequence(n_frames=400)
    np.testing.assert_array_equal(a.scene.boxes, b.scene.boxes)
    np.testing.assert_array_equal(np.stack(a.poses), np.stack(b.poses))
    pos = np.stack([T[:3, 3] for T in a.poses])
    step = np.linalg.norm(np.diff(pos[:, :2], axis=0), axis=1)
    assert 0.4 < step.min() and step.max() < 0.8                     # ~5-7 m/s at 10 Hz
    # no box footprint contains the sensor position (boxes are yaw-rotated rectangles)
    bx = a.scene.boxes
    for p in pos[::10]:
        c, s = np.cos(-bx[:, 6]), np.sin(-bx[:, 6])
        dx, dy = p[0] - bx[:, 0], p[1] - bx[:, 1]
        lx, ly = c * dx - s * dy, s * dx + c * dy
        inside = (np.abs(lx) <= bx[:, 3]) & (np.abs(ly) <= bx[:, 4]) & (p[2] <= 2 * bx[:, 5])
        assert not inside.any(), p


def test_xcd_block_order_is_a_bijection():
    """lo_kernels.hip xcd_block (XCD-aware logical block order), restated: a permutation of [0, nb) for any nb."""
    def xcd_block(h, nb, k=8):
        q, r, x, j = nb // k, nb % k, h % k, h // k
        return x * (q + 1) + j if x < r else r * (q + 1) + (x - r) * q + j
    for nb in (1, 7, 8, 9, 16, 100, 3907, 4096 * 16 + 3):
        got = sorted(xcd_block(h, nb) for h in range(nb))
        assert got == list(range(nb)), nb
