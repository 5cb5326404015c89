#!/bin/bash
# Copy the judged summaries of a scripts/profile_round.sh pass from gpurun_out/ into profiles/<tag>_*.
#   scripts/collect_profiles.sh r01
set -e
cd "$(dirname "$0")/.."
tag="$1"
[ -n "$tag" ] || { echo "usage: $0 <tag>"; exit 2; }
mkdir -p profiles
for w in kitti 1m kd e2e; do
    f=gpurun_out/stats_$w/run_kernel_stats.csv
    [ -f "$f" ] && cp "$f" "profiles/${tag}_${w}_kernel_stats.csv"
    t=gpurun_out/stats_$w/run_kernel_trace.csv
    [ -f "$t" ] && python scripts/trace_summary.py "$t" --out "profiles/${tag}_${w}_trace_summary.json" > /dev/null
    if [ -d gpurun_out/pmc_fetch_$w ] && [ -d gpurun_out/pmc_write_$w ]; then
        name=$w; [ "$w" = 1m ] && name=patch1m
        python scripts/pmc_summary.py --workload "$name" --fetch gpurun_out/pmc_fetch_$w \
            --write gpurun_out/pmc_write_$w --out profiles/pmc_traffic.json --note "$tag" > /dev/null
    fi
done
for b in kitti patch1m patch1m_random kitti_kdtree mid360 kitti_raw kitti_e2e kitti_loop; do
    [ -s gpurun_out/bench_$b.json ] && tail -n 1 gpurun_out/bench_$b.json > "profiles/${tag}_bench_$b.json"
done
[ -f gpurun_out/tests.log ] && tail -n 5 gpurun_out/tests.log > "profiles/${tag}_gpu_tests.txt"
ls -la profiles
