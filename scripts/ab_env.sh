#!/bin/bash
# A/B of two environment settings of the SAME library on one box (e.g. LO_PIPE=0 vs LO_PIPE=1): alternating short
# default-config bench runs, value per run into gpurun_out/ab.txt.   scripts/ab_env.sh "<envA>" "<envB>" [rounds]
A="$1"; B="$2"; R="${3:-2}"
mkdir -p gpurun_out
for r in $(seq "$R"); do
  for E in "$A" "$B"; do
    v=$(env $E timeout -k 10 300 python bench.py --no-cpu-baseline --pmc off --batch "" --sequences 0 \
        --steps 2000 --warmup 40 | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])") || exit 3
    echo "$E $v" | tee -a gpurun_out/ab.txt
  done
done
