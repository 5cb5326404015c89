"""Child process of tests/test_gpu_pipeline.py::test_pipeline_timeout_under_counter_collection (test infrastructure).

Run under `rocprofv3 --pmc FETCH_SIZE`, which serialises kernel dispatches across queues: the scan pipeline's
device-side waits (k_wait_final / k_wait_seq) can then wait for work that cannot start.  With LO_PIPE=1 forcing the
pipeline on and LO_PIPE_WAIT_MS bounding the waits, prints one JSON line: whether every synchronous result equals the
pipeline-off result bit for bit, whether every queued (async) record either equals it or reports LO_ERR_PIPELINE, and
lo_pipeline_status before / after."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.zeros(1, device="cuda")
    from tests import _data
    from tests.test_gpu_pipeline import _cases, _ctx, _queued, _run
    cs = _cases()[:6]
    o = _ctx(cs[0][0])
    L = o._L
    st0 = (C.c_int * 4)()
    L.lo_pipeline_status(o.ctx, st0)
    o.set_pipeline(False)
    ref = [_run(o, pts, Ti) for _, pts, Ti in cs]
    d_scans = [torch.from_numpy(np.ascontiguousarray(p, np.float32).reshape(-1, 3)).to("cuda:0") for _, p, _ in cs]
    inits = [Ti for _, _, Ti in cs]
    order = [k % len(cs) for k in range(12)]
    ref_q = _queued(o, d_scans, inits, order)
    on = bool(st0[0])                                      # the context's own default (LO_PIPE / counter collection)
    o.set_pipeline(on, 2)
    got_q = _queued(o, d_scans, inits, order)
    q_ok = all(np.array_equal(got_q[k].view(np.uint32), ref_q[k].view(np.uint32)) or int(got_q[k, 12]) == -5
               for k in range(len(order)))
    q_err = sum(int(got_q[k, 12]) == -5 for k in range(len(order)))
    o.set_pipeline(on, 2)
    sync_ok = all(_run(o, pts, Ti) == ref[j] for j, (_, pts, Ti) in enumerate(cs))
    st1 = (C.c_int * 4)()
    L.lo_pipeline_status(o.ctx, st1)
    o.close()
    print(json.dumps({"status_start": list(st0), "status_end": list(st1), "sync_bitwise": sync_ok,
                      "queued_bitwise_or_flagged": q_ok, "queued_flagged": q_err}), flush=True)


if __name__ == "__main__":
    main()
