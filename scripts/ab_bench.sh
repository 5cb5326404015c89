#!/bin/bash
# Same-box A/B of two or more builds of the library (box-to-box variance is a few %): alternating short
# default-config bench runs, value per run into gpurun_out/ab.txt.
#   scripts/ab_bench.sh <libA.so> <libB.so> [rounds]            (the historical two-library form)
#   AB_ROUNDS=R scripts/ab_bench.sh <lib1.so> <lib2.so> <lib3.so> ...
if [ $# -eq 3 ] && [[ "$3" =~ ^[0-9]+$ ]]; then LIBS=("$1" "$2"); R="$3"; else LIBS=("$@"); R="${AB_ROUNDS:-2}"; fi
mkdir -p gpurun_out
for r in $(seq "$R"); do
  for L in "${LIBS[@]}"; do
    v=$(LO_ICP_LIB="$L" timeout -k 10 300 python bench.py --no-cpu-baseline --pmc off --batch "" --sequences 0 \
        --steps 2000 --warmup 40 | python -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
m = d.get('roofline_dominant', {}).get('measured_live', {})
print(d['value'], 'gn_iter/scan %.4f' % (d['gn_iters_per_sec'] / d['value']),
      'cyc/EM-iter %.1f' % (m.get('cycles_per_em_iteration') or 0), 'EM-iter/fit %.2f' % (m.get('em_iterations_per_fit') or 0))
") || exit 3
    echo "$(basename "$L") $v" | tee -a gpurun_out/ab.txt
  done
done
