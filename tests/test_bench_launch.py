"""bench.py's multi-rank launcher (driver contract: `python bench.py --gpus N` with plain python).

Without WORLD_SIZE in the environment bench.py spawns N rank processes itself (RANK/LOCAL_RANK/WORLD_SIZE,
rendezvous on 127.0.0.1) before anything touches a GPU; a world size that disagrees with --gpus fails loudly.
`--dry-run` exercises that plumbing on CPU with gloo and no ICP: the gathered pose records of the last step must
equal every rank's own record, and the line must report n_gpus = N.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_spawn_two_ranks_dry_run():
    p = _run(["--gpus", "2", "--dry-run", "--steps", "30", "--warmup", "2"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout                       # exactly one JSON line, native prints went to stderr
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 30
    chk = d["gather_check"]
    assert chk["ranks"] == 2 and chk["records_equal"] is True
    assert len(d["per_rank_s"]) == 2


def test_world_size_mismatch_fails_loudly():
    p = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE=1 but --gpus 2" in p.stderr


def test_bad_gpu_count_rejected():
    p = _run(["--gpus", "0", "--dry-run"])
    assert p.returncode != 0
