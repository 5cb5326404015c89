#!/bin/bash
# Same-box A/B of library builds on the batched (multi-sequence) lines: value (single sequence) and the batched
# scans/s per B.   AB_ROUNDS=R scripts/ab_batch.sh <lib1.so> <lib2.so> ...      (results in gpurun_out/ab_batch.txt)
R="${AB_ROUNDS:-2}"
mkdir -p gpurun_out
for r in $(seq "$R"); do
  for L in "$@"; do
    v=$(LO_ICP_LIB="$L" timeout -k 10 300 python bench.py --no-cpu-baseline --pmc off --batch 1024,4096 --sequences 0 \
        --steps 300 --warmup 20 | python -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('%.1f' % d['value'], ' '.join('B=%d:%.0f' % (x['sequences'], x['value']) for x in d['batched']['runs']))
") || exit 3
    echo "$(basename "$L") $v" | tee -a gpurun_out/ab_batch.txt
  done
done
