"""Regenerate the voxel map's container iteration-order golden vectors from the REFERENCE's unordered_dense.

Builds an oracle VoxelMap (oracle/, the restated UpdateVoxelMap / ApplyTransformAndRehash) over KITTI-like keyframes
with its container-operation trace on, replays the trace on the real ankerl::unordered_dense 4.8.1 containers with
the reference's VoxelKeyHash (``oracle/_ref/map_order_golden``, compiled in place from the reference's vendored
header by ``make -C oracle ref``) and writes ``tests/golden/map_order_golden.npz``:

  kf_points (N, 3) float32, kf_offsets (K + 1,), kf_sensor (K, 3) float64, max_distance, planarity, transform (12,)
      the inputs: K keyframe world clouds (UpdateVoxelMap), then one ApplyTransformAndRehash(transform)
  cp<i>_l0 / cp<i>_l1 / cp<i>_cnt / cp<i>_ch   the real containers' iteration orders after update call i

A small pruning radius and the kitti.yaml planarity threshold make the sequence erase L0 voxels (radius pruning),
empty L1 voxels and whole non-planar L1 voxels with their children (erase-by-swap reorders the dense arrays).

Usage:  make -C oracle ref && python tests/golden/make_map_order_golden.py
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
DRIVER = os.path.join(ROOT, "oracle", "_ref", "map_order_golden")
sys.path.insert(0, ROOT)

MAX_DISTANCE = 25.0
PLANARITY = 0.1


def inputs():
    import oracle
    from lidar_odometry_amd import synth
    seq = synth.KittiLikeSequence(seed=7, n_frames=42)
    pts, offs, sens = [], [0], []
    for k in range(0, 40, 4):
        w = synth.transform(seq.poses[k], oracle.voxel_filter(seq.scan(k), 0.5, 8))
        pts.append(np.asarray(w, np.float32))
        offs.append(offs[-1] + len(w))
        sens.append(np.asarray(seq.poses[k][:3, 3], np.float64))
    T = synth.se3(synth.rot_z(0.02), [0.3, -0.2, 0.05])[:3].astype(np.float32).reshape(12)
    return np.concatenate(pts), np.asarray(offs, np.int64), np.stack(sens), T


def build_oracle(pts, offs, sens, T, trace=True):
    import oracle
    m = oracle.VoxelMap(0.5, 3, PLANARITY, True)
    if trace:
        m.enable_trace(True)
    states = []
    for k in range(len(sens)):
        m.update(pts[offs[k]:offs[k + 1]], sens[k], MAX_DISTANCE, True)
        states.append(m.orders())
    m.apply_transform(T)
    states.append(m.orders())
    return m, states


def replay(trace):
    with tempfile.TemporaryDirectory() as td:
        fi, fo = os.path.join(td, "t.bin"), os.path.join(td, "o.bin")
        np.ascontiguousarray(trace, np.int32).tofile(fi)
        subprocess.run([DRIVER, fi, fo], check=True)
        raw = np.fromfile(fo, np.int32)
    out, p = [], 0
    while p < len(raw):
        n0, n1, nc = raw[p:p + 3]
        p += 3
        l0 = raw[p:p + 3 * n0].reshape(-1, 3); p += 3 * n0
        l1 = raw[p:p + 3 * n1].reshape(-1, 3); p += 3 * n1
        cnt = raw[p:p + n1]; p += n1
        ch = raw[p:p + 3 * nc].reshape(-1, 3); p += 3 * nc
        out.append((l0, l1, cnt, ch))
    return out


def main():
    if not os.path.exists(DRIVER):
        sys.exit(f"{DRIVER} missing: run `make -C oracle ref` (needs /root/reference)")
    pts, offs, sens, T = inputs()
    m, _ = build_oracle(pts, offs, sens, T)
    tr = m.trace()
    real = replay(tr)
    arrays = {"kf_points": pts, "kf_offsets": offs, "kf_sensor": sens, "max_distance": np.float64(MAX_DISTANCE),
              "planarity": np.float32(PLANARITY), "transform": T}
    for i, (l0, l1, cnt, ch) in enumerate(real):
        arrays[f"cp{i}_l0"], arrays[f"cp{i}_l1"], arrays[f"cp{i}_cnt"], arrays[f"cp{i}_ch"] = l0, l1, cnt, ch
    ops = np.bincount(tr[:, 0], minlength=10)
    print(f"{len(sens)} keyframes + 1 rehash, {len(tr)} container ops: L0 ins {ops[1]} era {ops[2]}, L1 ins {ops[3]} "
          f"era {ops[4]}, child ins {ops[5]} era {ops[6]}; final L0 {len(real[-1][0])}, L1 {len(real[-1][1])}")
    np.savez_compressed(os.path.join(HERE, "map_order_golden.npz"), **arrays)


if __name__ == "__main__":
    main()
