"""Regenerate the PKO golden vectors from the REFERENCE implementation.

Runs ``oracle/_ref/pko_golden`` (the reference's own ``src/optimization/AdaptiveMEstimator.cpp``
compiled in place from /root/reference by ``make -C oracle ref``) on seeded residual vectors and writes

  tests/golden/pko_inputs.npz     residual vectors (inputs), keys case_<i>
  tests/golden/pko_golden.jsonl   reference outputs: alpha, GMM weights/means/variances, alpha grid, Z,
                                  std::shuffle(mt19937(42)) sample prefix and k-means seed draws
  tests/golden/pko_golden_kernels.jsonl  the same for the other pko_kernel_type values on a subset of the cases

Usage:  make -C oracle ref && python tests/golden/make_pko_golden.py
The fixtures are data only; the reference source never leaves /root/reference.
"""
from __future__ import annotations

import json
import os
import struct
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
DRIVER = os.path.join(ROOT, "oracle", "_ref", "pko_golden")


def cases():
    rng = np.random.default_rng(20251226)
    out = []
    # (name, vector) — normalised residuals r/scale as optimize() feeds them (>= 0)
    for n in (1, 2, 3, 5, 10, 50, 99, 100, 101, 257, 1000, 4001, 8000, 12000):
        out.append((f"halfnormal_{n}", np.abs(rng.normal(0.0, 6.0, n))))
    for n in (100, 999, 5000):
        inl = np.abs(rng.normal(0.0, 3.0, n))
        mask = rng.random(n) < 0.2
        inl[mask] = rng.uniform(0.0, 60.0, mask.sum())
        out.append((f"mixture_{n}", inl))
    out.append(("exponential_3000", rng.exponential(4.0, 3000)))
    out.append(("heavy_tail_2000", np.abs(rng.standard_cauchy(2000))))
    out.append(("all_equal_500", np.full(500, 3.0)))
    out.append(("mostly_zero_300", np.where(rng.random(300) < 0.9, 0.0, rng.uniform(0, 5, 300))))
    out.append(("two_values_200", np.where(rng.random(200) < 0.5, 1.0, 7.0)))
    # realistic: |n.(p-c)| in metres, normalised by std/6 of the same vector
    r = np.abs(rng.normal(0.0, 0.05, 9000))
    r[rng.random(9000) < 0.1] = rng.uniform(0, 1.0, int((rng.random(9000) < 0.1).sum()))[: int((rng.random(9000) < 0.1).sum())].mean()
    r = np.abs(r)
    scale = np.sqrt(np.mean((r - r.mean()) ** 2)) / 6.0
    out.append(("icp_like_9000", r / scale))
    # shuffle mode boundaries (libstdc++ pairs draws for n <= 65535)
    for n in (65535, 65536, 70001):
        out.append((f"halfnormal_{n}", np.abs(rng.normal(0.0, 6.0, n))))
    return out


# pko_kernel_type values of AdaptiveMEstimator.cpp:128-156 besides kitti.yaml's "huber"; "robust" is not a kernel
# name, so the reference falls back to Cauchy for it.  Run on a subset of the cases.
KERNELS = ("cauchy", "tukey", "welsch", "gemanMcClure", "pseudoHuber", "robust")
KERNEL_CASES = ("halfnormal_100", "halfnormal_1000", "mixture_999", "exponential_3000", "heavy_tail_2000",
                "icp_like_9000", "halfnormal_12000")


def _write_inputs(path, vecs):
    with open(path, "wb") as f:
        f.write(struct.pack("<i", len(vecs)))
        for v in vecs:
            v = np.ascontiguousarray(v, dtype="<f8")
            f.write(struct.pack("<i", len(v)))
            f.write(v.tobytes())


def main():
    if not os.path.exists(DRIVER):
        sys.exit(f"missing {DRIVER}: run `make -C oracle ref` (needs /root/reference)")
    cs = cases()
    inp = os.path.join(HERE, "_pko_in.bin")
    outp = os.path.join(HERE, "pko_golden.jsonl")
    _write_inputs(inp, [v for _, v in cs])
    subprocess.run([DRIVER, inp, outp], check=True, stdout=subprocess.DEVNULL)
    # the other PKO kernels: one JSON line per (kernel, case), "case" indexing pko_inputs.npz
    names = [c[0] for c in cs]
    sel = [names.index(n) for n in KERNEL_CASES]
    _write_inputs(inp, [cs[i][1] for i in sel])
    tmp = os.path.join(HERE, "_pko_kernel.jsonl")
    with open(os.path.join(HERE, "pko_golden_kernels.jsonl"), "w") as out:
        for kern in KERNELS:
            subprocess.run([DRIVER, inp, tmp, kern], check=True, stdout=subprocess.DEVNULL)
            with open(tmp) as f:
                for j, line in enumerate(f):
                    rec = json.loads(line)
                    rec["case"] = sel[j]
                    rec["name"] = names[sel[j]]
                    rec["kernel"] = kern
                    out.write(json.dumps(rec) + "\n")
    os.remove(tmp)
    os.remove(inp)
    np.savez_compressed(os.path.join(HERE, "pko_inputs.npz"),
                        names=np.array([c[0] for c in cs]),
                        **{f"case_{i}": c[1] for i, c in enumerate(cs)})
    print(f"wrote {len(cs)} cases -> {outp}")


if __name__ == "__main__":
    main()
