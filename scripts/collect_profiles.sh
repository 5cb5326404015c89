#!/bin/bash
# Copy the judged summaries of a scripts/profile_round.sh pass from gpurun_out/ into profiles/<tag>_*.
#   scripts/collect_profiles.sh r01
set -e
cd "$(dirname "$0")/.."
tag="$1"
[ -n "$tag" ] || { echo "usage: $0 <tag>"; exit 2; }
mkdir -p profiles
for w in kitti 1m kd e2e loop; do
    f=gpurun_out/summ/${w}_kernel_stats.csv
    [ -f "$f" ] && cp "$f" "profiles/${tag}_${w}_kernel_stats.csv"
    t=gpurun_out/summ/${w}_trace_summary.json
    [ -f "$t" ] && cp "$t" "profiles/${tag}_${w}_trace_summary.json"
done
[ -f gpurun_out/summ/pmc_traffic.json ] && cp gpurun_out/summ/pmc_traffic.json profiles/pmc_traffic.json
for b in kitti patch1m patch1m_random kitti_kdtree mid360 kitti_raw kitti_e2e kitti_loop; do
    [ -s gpurun_out/bench_$b.json ] && tail -n 1 gpurun_out/bench_$b.json > "profiles/${tag}_bench_$b.json"
done
[ -f gpurun_out/tests.log ] && tail -n 5 gpurun_out/tests.log > "profiles/${tag}_gpu_tests.txt"
ls -la profiles
