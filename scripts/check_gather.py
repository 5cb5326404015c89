"""Rehearsal of the scan-parallel pose gather (parallel.PipelinedPoseGather) with real collectives on GPU tensors.

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 scripts/check_gather.py [nccl|gloo]

Every rank writes rank * 1000 + step into its ring slot on the main stream and gathers it on the side stream;
the last `depth` steps' gathered records must hold every rank's value.  On a one-GPU box all ranks share cuda:0
(RCCL may refuse two ranks on one device; the script then reports that and exits 3)."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lidar_odometry_amd.parallel import PipelinedPoseGather  # noqa: E402


def main():
    backend = sys.argv[1] if len(sys.argv) > 1 else "nccl"
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ngpu = torch.cuda.device_count()
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(ngpu, 1))
    torch.cuda.set_device(dev)
    try:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        pg = PipelinedPoseGather(world, dev, depth=4)
        steps = 64
        for k in range(steps):
            s = pg.slot()
            s.fill_(float(rank * 1000 + k))
            # some main-stream work between steps (the ICP kernels' place)
            x = torch.ones(1 << 16, device=dev)
            for _ in range(4):
                x = x * 1.0001
            pg.launch()
        torch.cuda.synchronize(dev)
        bad = 0
        for k in range(steps - 4, steps):
            r = pg.records(k)
            for q in range(world):
                if not (r[q] == q * 1000 + k).all():
                    bad += 1
        print(f"[rank {rank}] backend {backend} world {world} on {dev}: {'OK' if bad == 0 else f'{bad} BAD records'}",
              flush=True)
        dist.barrier()
        dist.destroy_process_group()
        sys.exit(0 if bad == 0 else 1)
    except Exception as e:  # noqa: BLE001
        print(f"[rank {rank}] backend {backend}: {type(e).__name__}: {e}", flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
