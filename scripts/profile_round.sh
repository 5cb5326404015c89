#!/bin/bash
# One measurement pass on the GPU box (run from the repo root under gpurun):
#   parity tests, bench lines (kitti default + patch1m), rocprofv3 kernel stats, and separate PMC passes
#   (FETCH_SIZE, WRITE_SIZE) for the HBM-traffic figure.  Everything lands in gpurun_out/; copy the
#   summaries into profiles/<tag>_* afterwards (scripts/collect_profiles.sh <tag>).
#   scripts/profile_round.sh [skip_tests]
cd "$(dirname "$0")/.." || exit 2
steps=()
if [ "$1" != "skip_tests" ]; then
    steps+=("tests:900:python -m pytest tests -m gpu -x -q -p no:cacheprovider")
fi
steps+=(
  "bench_kitti:600:python bench.py > gpurun_out/bench_kitti.json"
  "bench_1m:900:python bench.py --config patch1m --steps 40 --warmup 4 --cpu-budget 10 > gpurun_out/bench_patch1m.json"
  "bench_1m_rand:600:python bench.py --config patch1m --order random --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/bench_patch1m_random.json"
  "bench_kd:600:python bench.py --config kitti_kdtree --cpu-budget 10 > gpurun_out/bench_kitti_kdtree.json"
  "bench_mid360:600:python bench.py --config mid360 --cpu-budget 10 > gpurun_out/bench_mid360.json"
  "stats_kd:600:rocprofv3 --kernel-trace --stats -d gpurun_out/stats_kd -o run --output-format csv -- python bench.py --config kitti_kdtree --steps 200 --warmup 10 --no-cpu-baseline"
  "stats_kitti:600:rocprofv3 --kernel-trace --stats -d gpurun_out/stats_kitti -o run --output-format csv -- python bench.py --steps 200 --warmup 10 --no-cpu-baseline"
  "stats_1m:600:rocprofv3 --kernel-trace --stats -d gpurun_out/stats_1m -o run --output-format csv -- python bench.py --config patch1m --steps 20 --warmup 2 --no-cpu-baseline"
  "pmcf_kitti:600:rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_kitti -o run --output-format csv -- python bench.py --steps 200 --warmup 10 --no-cpu-baseline"
  "pmcw_kitti:600:rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_kitti -o run --output-format csv -- python bench.py --steps 200 --warmup 10 --no-cpu-baseline"
  "pmcf_1m:600:rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_1m -o run --output-format csv -- python bench.py --config patch1m --steps 20 --warmup 2 --no-cpu-baseline"
  "pmcw_1m:600:rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_1m -o run --output-format csv -- python bench.py --config patch1m --steps 20 --warmup 2 --no-cpu-baseline"
)
exec scripts/gpu_steps.sh "${steps[@]}"
