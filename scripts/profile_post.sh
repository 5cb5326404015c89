#!/bin/bash
# Summarise the raw rocprofv3 output of scripts/profile_round.sh into gpurun_out/summ/ and delete the raw CSVs
# (kernel traces of the batched runs are hundreds of MB; gpurun merges at most 64 MiB back).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out/summ
cp profiles/pmc_traffic.json gpurun_out/summ/pmc_traffic.json
for w in kitti 1m kd e2e loop; do
    d=gpurun_out/stats_$w
    [ -f "$d/run_kernel_stats.csv" ] && cp "$d/run_kernel_stats.csv" "gpurun_out/summ/${w}_kernel_stats.csv"
    [ -f "$d/run_kernel_trace.csv" ] && python scripts/trace_summary.py "$d/run_kernel_trace.csv" \
        --out "gpurun_out/summ/${w}_trace_summary.json" > /dev/null
    if [ -d gpurun_out/pmc_fetch_$w ] && [ -d gpurun_out/pmc_write_$w ]; then
        name=$w; [ "$w" = 1m ] && name=patch1m
        python scripts/pmc_summary.py --workload "$name" --fetch gpurun_out/pmc_fetch_$w \
            --write gpurun_out/pmc_write_$w --out gpurun_out/summ/pmc_traffic.json --note "${PROFILE_TAG:-r02}" > /dev/null
    fi
done
rm -rf gpurun_out/stats_* gpurun_out/pmc_fetch_* gpurun_out/pmc_write_*
ls -la gpurun_out/summ
