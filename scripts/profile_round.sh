#!/bin/bash
# One measurement pass on the GPU box (run from the repo root under gpurun):
#   parity tests, bench lines (kitti default + patch1m), rocprofv3 kernel stats, and separate PMC passes
#   (FETCH_SIZE, WRITE_SIZE) for the HBM-traffic figure.  Everything lands in gpurun_out/; copy the
#   summaries into profiles/<tag>_* afterwards (scripts/collect_profiles.sh <tag>).
#   scripts/profile_round.sh [step names...]      (no names: every step; gpurun's 1200 s cap usually needs two calls)
cd "$(dirname "$0")/.." || exit 2
all=(
  "tests:900:python -m pytest tests -m gpu -x -q -p no:cacheprovider"
  "bench_kitti:600:python bench.py > gpurun_out/bench_kitti.json"
  "pko_phases:300:python scripts/pko_phases.py > gpurun_out/pko_phases.txt"
  "bench_1m:900:python bench.py --config patch1m --steps 40 --warmup 4 --cpu-budget 10 > gpurun_out/bench_patch1m.json"
  "bench_1m_rand:600:python bench.py --config patch1m --order random --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/bench_patch1m_random.json"
  "bench_raw:600:python bench.py --config kitti_raw --cpu-budget 10 > gpurun_out/bench_kitti_raw.json"
  "bench_e2e:900:python bench.py --config kitti_e2e --steps 600 --cpu-budget 15 > gpurun_out/bench_kitti_e2e.json"
  "bench_loop:600:python bench.py --config kitti_loop --steps 200 --warmup 12 --cpu-budget 10 > gpurun_out/bench_kitti_loop.json"
  "bench_kd:600:python bench.py --config kitti_kdtree --cpu-budget 10 > gpurun_out/bench_kitti_kdtree.json"
  "bench_mid360:600:python bench.py --config mid360 --cpu-budget 10 > gpurun_out/bench_mid360.json"
  "stats_kd:600:rocprofv3 --kernel-trace --stats -d gpurun_out/stats_kd -o run --output-format csv -- python bench.py --config kitti_kdtree --steps 200 --warmup 10 --no-cpu-baseline --pmc off"
  "stats_kitti:600:rocprofv3 --kernel-trace --stats -d gpurun_out/stats_kitti -o run --output-format csv -- python bench.py --steps 200 --warmup 10 --no-cpu-baseline --pmc off --batch 1024 --sequences 0"
  "stats_e2e:600:rocprofv3 --kernel-trace --stats -d gpurun_out/stats_e2e -o run --output-format csv -- python bench.py --config kitti_e2e --steps 240 --no-cpu-baseline --pmc off"
  "stats_loop:600:rocprofv3 --kernel-trace --stats -d gpurun_out/stats_loop -o run --output-format csv -- python bench.py --config kitti_loop --steps 100 --warmup 12 --no-cpu-baseline --pmc off"
  "stats_1m:600:rocprofv3 --kernel-trace --stats -d gpurun_out/stats_1m -o run --output-format csv -- python bench.py --config patch1m --steps 20 --warmup 2 --no-cpu-baseline --pmc off"
  "pmcf_kitti:600:LO_PIPE=0 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_kitti -o run --output-format csv -- python bench.py --steps 200 --warmup 10 --no-cpu-baseline --pmc off"
  "pmcw_kitti:600:LO_PIPE=0 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_kitti -o run --output-format csv -- python bench.py --steps 200 --warmup 10 --no-cpu-baseline --pmc off"
  "pmcf_1m:600:rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_1m -o run --output-format csv -- python bench.py --config patch1m --steps 20 --warmup 2 --no-cpu-baseline --pmc off"
  "pmcw_1m:600:rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_1m -o run --output-format csv -- python bench.py --config patch1m --steps 20 --warmup 2 --no-cpu-baseline --pmc off"
)
# post: summaries of the traces / PMC passes into gpurun_out/summ/, then the raw CSVs are deleted (gpurun merges
# at most 64 MiB of gpurun_out/ back)
all+=("post:300:scripts/profile_post.sh")
steps=()
for spec in "${all[@]}"; do
    if [ $# -eq 0 ]; then steps+=("$spec"); continue; fi
    for want in "$@"; do [ "${spec%%:*}" = "$want" ] && steps+=("$spec"); done
done
exec scripts/gpu_steps.sh "${steps[@]}"
