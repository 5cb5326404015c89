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


def all_ranks_agree(flag: bool, world: int, device=None) -> bool:
    """True only if `flag` holds on every rank: one all-reduce (MIN) of a 0/1 int.  bench.py's --mode auto takes the
    fast arithmetic only when every rank's own parity check passed, so all ranks time the same mode (the per-rank
    parity verdicts stay in the line).  world == 1 needs no process group."""
    if world == 1:
        return bool(flag)
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()))


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


class PipelinedPoseGather:
    """The per-step pose all-gather taken off the critical path: step k's record is exported into ring slot
    k % depth and gathered on a side stream, so the next scans' ICP kernels on the main stream do not wait for
    the collective (a ~220 us KITTI scan would otherwise pay the collective's latency every step).  The main
    stream only waits when it is about to overwrite a slot whose gather has not finished (depth steps later).
    On CPU tensors (gloo) there are no streams and the gather runs in place.

        rec = pg.slot()          # export this step's record into rec (on the main stream)
        pg.launch()              # gather it on the side stream
        ...
        pg.drain(); pg.records(k)   # [world, 16] of step k (valid for the last `depth` steps)"""

    def __init__(self, world: int, device=None, depth: int = 4):
        import torch
        self.world, self.depth, self.k = world, depth, 0
        dev = torch.device(device) if device is not None else torch.device("cpu")
        self.recs = torch.zeros(depth, RECORD_FLOATS, dtype=torch.float32, device=dev)
        self.outs = torch.zeros(depth, RECORD_FLOATS * world, dtype=torch.float32, device=dev)
        self.cuda = dev.type == "cuda"
        self.side = torch.cuda.Stream(dev) if (self.cuda and world > 1) else None
        self.done = [None] * depth

    def slot(self):
        import torch
        i = self.k % self.depth
        if self.done[i] is not None:
            torch.cuda.current_stream(self.recs.device).wait_event(self.done[i])
        return self.recs[i]

    def launch(self):
        i = self.k % self.depth
        self.k += 1
        if self.world == 1:
            self.outs[i].copy_(self.recs[i])
            return
        import torch
        import torch.distributed as dist
        if self.side is None:
            dist.all_gather_into_tensor(self.outs[i], self.recs[i])
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.recs.device))
        with torch.cuda.stream(self.side):
            self.side.wait_event(ev)
            dist.all_gather_into_tensor(self.outs[i], self.recs[i])
            d = torch.cuda.Event()
            d.record(self.side)
            self.done[i] = d

    def drain(self):
        if self.side is not None:
            self.side.synchronize()

    def records(self, step: int) -> np.ndarray:
        if not (self.k - self.depth <= step < self.k):
            raise IndexError(f"step {step} is not in the ring (steps {self.k - self.depth}..{self.k - 1})")
        return self.outs[step % self.depth].detach().cpu().numpy().reshape(self.world, RECORD_FLOATS)


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
