"""Scan-parallel driver (lidar_odometry_amd/parallel.py) over world_size-2 gloo on CPU.

Each rank runs its round-robin share of KITTI-like scans through a per-rank optimizer and all-gathers the
16-float pose records; every rank must end with the same records a single process produces.  The per-rank
optimizer here is the CPU oracle (test infrastructure), so the collective / sharding logic is what is tested;
the GPU path through the same driver is exercised by bench.py --gpus N.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from lidar_odometry_amd import parallel

FRAMES = [11, 13, 17, 21, 25]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _records_single():
    import oracle
    from tests import _data
    out = []
    for f in FRAMES:
        m, pts, Ti, _ = _data.kitti_case(f)
        ok, To, it, logs = oracle.icp_optimize(m, pts, Ti)
        out.append(parallel.make_record(ok, To, it, logs[0]["n_corr"] if logs else 0))
    return np.stack(out)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from tests import _data

        def one(k):
            m, pts, Ti, _ = _data.kitti_case(FRAMES[k])
            ok, To, it, logs = oracle.icp_optimize(m, pts, Ti)
            return parallel.make_record(ok, To, it, logs[0]["n_corr"] if logs else 0)

        recs = parallel.run_replicas(one, len(FRAMES), rank, world)
        # the pipelined (ring) gather over the same steps: every step's gathered records equal the plain gather's
        import torch
        pg = parallel.PipelinedPoseGather(world, depth=2)
        piped = np.zeros_like(recs)
        for st in range(parallel.steps_for(len(FRAMES), world)):
            k = parallel.scan_of(st, rank, world)
            pg.slot().copy_(torch.as_tensor(one(min(k, len(FRAMES) - 1))))
            pg.launch()
            pg.drain()
            g = pg.records(st)
            for r in range(world):
                kk = parallel.scan_of(st, r, world)
                if kk < len(FRAMES):
                    piped[kk] = g[r]
        q.put((rank, recs, piped))
    finally:
        dist.destroy_process_group()


def _agree_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # bench.py --mode auto: a rank whose own parity check failed keeps every rank on reference-exact
        q.put((rank, [parallel.all_ranks_agree(f, world) for f in
                      ([True, rank == 0, rank == 1, False])]))
    finally:
        dist.destroy_process_group()


def test_mode_agreement_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == got[1] == [True, False, False, False]
    assert parallel.all_ranks_agree(True, 1) and not parallel.all_ranks_agree(False, 1)


def test_assignment_covers_all_scans():
    for n in (1, 2, 5, 8, 17):
        for w in (1, 2, 3, 8):
            got = sorted(k for r in range(w) for k in parallel.scan_assignment(n, r, w))
            assert got == list(range(n))
            assert parallel.steps_for(n, w) == max(len(parallel.scan_assignment(n, r, w)) for r in range(w))


def test_single_rank_no_process_group():
    import torch
    g = parallel.PoseAllGather(1)
    t = torch.arange(16, dtype=torch.float32)
    assert g(t) is t


def test_pipelined_gather_single_rank_ring():
    import torch
    pg = parallel.PipelinedPoseGather(1, depth=3)
    for k in range(7):
        pg.slot().fill_(float(k))
        pg.launch()
    pg.drain()
    for k in range(4, 7):
        assert (pg.records(k) == k).all()
    with pytest.raises(IndexError):
        pg.records(3)
    assert torch.is_tensor(pg.slot())


def test_scan_parallel_gloo_world2():
    ref = _records_single()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, recs, piped = q.get(timeout=300)
        res[r] = recs
        np.testing.assert_array_equal(piped, recs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        np.testing.assert_array_equal(res[r], ref)
    poses = parallel.gathered_poses(res[0])
    assert poses.shape == (len(FRAMES), 3, 4)
    assert (res[0][:, 12] == 0).all()          # all scans converged with enough correspondences
