"""Instruction mix of the split-EM loop of k_pko_t (one EM iteration of one component wave) from the gfx950 ISA.

    python scripts/pko_em_isa.py [--spl 2] [--k 3]

Compiles lidar_odometry_amd/csrc/lo_pko.hip to assembly, finds the EM loops of the single-scan kernel (loop bodies
holding the per-iteration s_barrier and the permlane butterfly) and counts their instructions by class.  With the
per-class issue costs measured by scripts/lat_bench.hip on MI355X this gives the EM iteration's issue floor, the
latency roofline of the dominant kernel (profiles/pko_latency.json)."""
import argparse
import collections
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def classify(op: str) -> str:
    if op in ("v_rcp_f64_e32", "v_rsq_f64_e32", "v_sqrt_f64_e32"):
        return "fp64_trans"
    if re.match(r"v_(fma|fmac|mul|add|max|min|ldexp|rndne|cvt_i32|cvt_f64|frexp|fract|cmp\w*)_f64", op) or \
            re.match(r"v_\w+_f64", op):
        return "fp64"
    if "permlane" in op:
        return "permlane"
    if "_dpp" in op or op.startswith("v_mov_b32_dpp"):
        return "dpp"
    if op.startswith("v_readlane") or op.startswith("v_readfirstlane"):
        return "readlane"
    if op.startswith("ds_"):
        return "lds"
    if op == "s_barrier":
        return "barrier"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu32"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hipcc", default="/opt/rocm/bin/hipcc")
    args = ap.parse_args()
    src = os.path.join(ROOT, "lidar_odometry_amd", "csrc", "lo_pko.hip")
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "pko.s")
        subprocess.run([args.hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "--offload-device-only", "-S", "-o", out, src], check=True, capture_output=True)
        lines = open(out).read().split("\n")
    # the single-scan kernel only
    start = next(i for i, l in enumerate(lines) if re.match(r"^_ZN2lo7k_pko_tILi4EEEvNS_7KParamsEii:", l))
    end = next(i for i in range(start + 1, len(lines)) if re.match(r"^_Z\w+:", lines[i]))
    body = lines[start:end]
    # loop membership from the compiler's block comments: "; =>This (Inner) Loop Header: Depth=d" opens loop BB, and
    # "; in Loop: Header=BB" (or "Parent Loop BB") marks a block of it; instructions are attributed to their block
    cur = None
    members = collections.defaultdict(list)
    for l in body:
        m = re.match(r"^\.(LBB\d+_\d+):(.*)$", l)
        if m:
            lab, com = m.group(1), m.group(2)
            h = re.search(r"Loop Header", com)
            h2 = re.search(r"Header=(BB\d+_\d+)", com)
            cur = ("L" + lab[1:]) if h else (("L" + h2.group(1)) if h2 else None)
            continue
        if cur and l.strip() and not l.strip().startswith((";", ".")):
            members[cur].append(l.split()[0])
    for lab, ops in members.items():
        cnt = collections.Counter(classify(o) for o in ops)
        if cnt["barrier"] == 0 or cnt["permlane"] == 0:
            continue
        rnd = sum(1 for o in ops if o.startswith("v_rndne_f64"))
        print(f"{lab}: {len(ops)} instructions, exps per lane {rnd}: " + ", ".join(f"{k} {v}" for k, v in sorted(cnt.items())))


if __name__ == "__main__":
    main()
