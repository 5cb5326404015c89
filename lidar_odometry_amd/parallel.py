"""Scan-parallel multi-GPU driver: one process per GPU, no map sharding.

The ICP step does not shard inside a scan (every GN iteration ends in a global 28-value reduction, PKO and a
6x6 solve), and consecutive scans of one sequence are sequential (the initial guess is the previous pose,
Estimator.cpp:154).  Ranks therefore run independent replicas: each owns its own map and scan stream, and the
only collective is an all-gather of one 16-float pose/status record per rank per step
(pose[12], status, iterations, n_corr, 0 -- the layout lo_icp_export_pose writes), over RCCL on GPUs
(backend "nccl") or gloo on CPU.

Scan k of a shared scan list goes to rank k % world at step k // world, so the gathered record of rank r
at step s belongs to scan s * world + r without carrying an index.
"""
from __future__ import annotations

from typing import Callable, List, Sequence

import numpy as np

RECORD_FLOATS = 16


def scan_assignment(n_scans: int, rank: int, world: int) -> List[int]:
    """Scan indices processed by `rank`, in step order (round-robin)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    return list(range(rank, n_scans, world))


def steps_for(n_scans: int, world: int) -> int:
    """Steps every rank runs so that all scans are covered (ranks past the end repeat their last scan)."""
    return (n_scans + world - 1) // world


def scan_of(step: int, rank: int, world: int) -> int:
    return step * world + rank


class PoseAllGather:
    """All-gather of one RECORD_FLOATS record per rank into a preallocated [world * 16] tensor.

    world == 1 needs no process group and returns the record itself."""

    def __init__(self, world: int, device=None):
        import torch
        self.world = world
        self.out = torch.zeros(RECORD_FLOATS * world, dtype=torch.float32, device=device)

    def __call__(self, rec):
        if self.world == 1:
            return rec
        import torch.distributed as dist
        dist.all_gather_into_tensor(self.out, rec)
        return self.out


def make_record(ok: bool, T34, iterations: int, n_corr: int) -> np.ndarray:
    """Host-side record in lo_icp_export_pose's layout (status: 0 = LO_OK, 1 = LO_INSUFFICIENT)."""
    r = np.zeros(RECORD_FLOATS, np.float32)
    r[:12] = np.asarray(T34, np.float32).reshape(12)
    r[12] = 0.0 if ok else 1.0
    r[13] = float(iterations)
    r[14] = float(n_corr)
    return r


def run_replicas(optimize_one: Callable[[int], np.ndarray], n_scans: int, rank: int, world: int,
                 device=None) -> np.ndarray:
    """Run scans round-robin over ranks; `optimize_one(scan_index)` returns this rank's 16-float record.

    Returns the gathered records of all scans, [n_scans, 16], identical on every rank."""
    import torch
    gather = PoseAllGather(world, device)
    out = np.zeros((n_scans, RECORD_FLOATS), np.float32)
    for s in range(steps_for(n_scans, world)):
        k = scan_of(s, rank, world)
        rec = optimize_one(min(k, n_scans - 1))
        t = torch.as_tensor(np.asarray(rec, np.float32), device=device)
        g = gather(t).detach().cpu().numpy().reshape(world, RECORD_FLOATS)
        for r in range(world):
            kk = scan_of(s, r, world)
            if kk < n_scans:
                out[kk] = g[r]
    return out


def gathered_poses(records: Sequence[np.ndarray]) -> np.ndarray:
    """[n, 3, 4] poses from gathered records."""
    a = np.asarray(records, np.float32).reshape(-1, RECORD_FLOATS)
    return a[:, :12].reshape(-1, 3, 4)
