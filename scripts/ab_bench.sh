#!/bin/bash
# A/B of two builds of the library on ONE box (box-to-box variance is a few %): alternating short default-config
# bench runs, value per run into gpurun_out/ab.txt.   scripts/ab_bench.sh <libA.so> <libB.so> [rounds] [extra env]
A="$1"; B="$2"; R="${3:-2}"
mkdir -p gpurun_out
for r in $(seq "$R"); do
  for L in "$A" "$B"; do
    v=$(LO_ICP_LIB="$L" timeout -k 10 300 python bench.py --no-cpu-baseline --pmc off --batch "" --sequences 0 \
        --steps 2000 --warmup 40 | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])") || exit 3
    echo "$(basename "$L") $v" | tee -a gpurun_out/ab.txt
  done
done
