"""Regenerate the 5-NN golden vectors of the KDTree correspondence variant from the REFERENCE's nanoflann.

Runs ``oracle/_ref/knn_golden`` (the reference's vendored ``thirdparty/nanoflann/nanoflann.hpp`` 1.7.1, configured
as ``util::KdTree`` -- PointCloudUtils.h:370-423 -- and compiled in place by ``make -C oracle ref``) on seeded
clouds and queries and writes ``tests/golden/knn_golden.npz``:

  <case>_cloud   (m, 3) float32   the map cloud (VoxelMap::GetPointCloud order)
  <case>_query   (q, 3) float32   query points (world frame, as find_correspondences_kdtree issues them)
  <case>_idx     (q, 5) int32     nanoflann's knnSearch indices (-1 past `found`)
  <case>_dist    (q, 5) float32   its fp32 squared distances (inf past `found`)
  <case>_found   (q,)   int32

Cases: the L0 centroid cloud of the bench's KITTI-like map (real query distribution: a scan at a perturbed pose),
integer lattices with queries on lattice points / cell centres / face centres (many exact fp32 distance ties, so
the visit-order tie-break is exercised), duplicated points, a tiny cloud (< 5 points), far-away and non-finite
queries.

Usage:  make -C oracle ref && python tests/golden/make_knn_golden.py
"""
from __future__ import annotations

import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
DRIVER = os.path.join(ROOT, "oracle", "_ref", "knn_golden")
sys.path.insert(0, ROOT)


def run_nanoflann(cloud, queries, k=5):
    cloud = np.ascontiguousarray(cloud, np.float32).reshape(-1, 3)
    queries = np.ascontiguousarray(queries, np.float32).reshape(-1, 3)
    with tempfile.TemporaryDirectory() as td:
        fi, fo = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(fi, "wb") as f:
            f.write(struct.pack("<i", len(cloud)))
            f.write(cloud.tobytes())
            f.write(struct.pack("<i", len(queries)))
            f.write(queries.tobytes())
            f.write(struct.pack("<i", k))
        subprocess.run([DRIVER, fi, fo], check=True)
        raw = np.fromfile(fo, dtype=np.uint8)
    rec = np.dtype([("found", "<i4"), ("idx", "<u4", (k,)), ("dist", "<f4", (k,))])
    out = raw.view(rec)
    idx = out["idx"].astype(np.int64)
    idx[idx == 0xFFFFFFFF] = -1
    return idx.astype(np.int32), out["dist"].astype(np.float32), out["found"].astype(np.int32)


def lattice(n, spacing=1.0, origin=(0.0, 0.0, 0.0)):
    g = np.arange(n, dtype=np.float32) * np.float32(spacing)
    x, y, z = np.meshgrid(g, g, g, indexing="ij")
    return (np.stack([x.ravel(), y.ravel(), z.ravel()], 1) + np.asarray(origin, np.float32)).astype(np.float32)


def cases():
    rng = np.random.default_rng(7)
    out = {}
    # 1. the KITTI-like bench map's L0 centroids and a scan through a perturbed pose (the production distribution)
    import bench
    from lidar_odometry_amd import synth
    wl = bench.build_kitti(0)
    cloud = wl["vm"].l0_cloud()
    q = synth.transform(wl["inits"][3], wl["scans"][3])
    out["kitti"] = (cloud, q[:2000])
    # 2. integer lattice, queries on lattice points, cell centres, face and edge centres: many exact ties
    L = lattice(12)
    perm = rng.permutation(len(L))                      # a shuffled insertion order, as a hash map would give
    Lp = L[perm]
    qs = [L[rng.integers(0, len(L), 200)],
          L[rng.integers(0, len(L), 200)] + np.float32(0.5),
          L[rng.integers(0, len(L), 200)] + np.array([0.5, 0.0, 0.0], np.float32),
          L[rng.integers(0, len(L), 200)] + np.array([0.5, 0.5, 0.0], np.float32)]
    out["lattice"] = (Lp, np.concatenate(qs).astype(np.float32))
    # 3. anisotropic lattice at 0.25 m (binary-exact coordinates), offsets that tie across split planes
    A = lattice(10, 0.25, (-1.0, 3.0, 0.5))
    A = A[rng.permutation(len(A))]
    qa = A[rng.integers(0, len(A), 300)] + rng.integers(-2, 3, (300, 3)).astype(np.float32) * np.float32(0.125)
    out["lattice_quarter"] = (A, qa.astype(np.float32))
    # 4. duplicated points (equal coordinates at different indices)
    D = rng.normal(0, 2.0, (300, 3)).astype(np.float32)
    D = np.concatenate([D, D[:120], D[50:80]])
    D = D[rng.permutation(len(D))]
    out["duplicates"] = (D, np.concatenate([D[:150], rng.normal(0, 2.0, (150, 3)).astype(np.float32)]))
    # 5. random planar patches (surface-like), queries near and far
    P = rng.uniform(-20, 20, (3000, 3)).astype(np.float32)
    P[:, 2] = np.round(P[:, 2] * 4) / 4
    out["patches"] = (P, np.concatenate([P[rng.integers(0, 3000, 300)] + rng.normal(0, 0.3, (300, 3)).astype(np.float32),
                                          rng.uniform(-500, 500, (50, 3)).astype(np.float32)]))
    # 6. fewer than 5 points, and non-finite queries
    T = rng.normal(0, 1, (4, 3)).astype(np.float32)
    out["tiny"] = (T, rng.normal(0, 1, (20, 3)).astype(np.float32))
    bad = np.array([[np.nan, 0, 0], [np.inf, 1, 2], [0, -np.inf, 0], [1e30, 1e30, 1e30]], np.float32)
    out["nonfinite"] = (Lp, bad)
    return out


def main():
    if not os.path.exists(DRIVER):
        sys.exit(f"{DRIVER} missing: run `make -C oracle ref` (needs /root/reference)")
    arrays = {}
    for name, (cloud, q) in cases().items():
        idx, dist, found = run_nanoflann(cloud, q)
        arrays[f"{name}_cloud"] = np.ascontiguousarray(cloud, np.float32)
        arrays[f"{name}_query"] = np.ascontiguousarray(q, np.float32)
        arrays[f"{name}_idx"] = idx
        arrays[f"{name}_dist"] = dist
        arrays[f"{name}_found"] = found
        ties = int(np.sum(dist[:, :4] == dist[:, 1:]))
        print(f"{name}: cloud {len(cloud)}, queries {len(q)}, found<5: {int(np.sum(found < 5))}, adjacent ties {ties}")
    np.savez_compressed(os.path.join(HERE, "knn_golden.npz"), **arrays)


if __name__ == "__main__":
    main()
