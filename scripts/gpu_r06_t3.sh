# Round 6: the exact solve's latency parts (microbenchmark), the split device-count scale kernels (tests + raw bench)
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 60 scripts/solve_microbench > gpurun_out/r06_solve_microbench.txt 2>&1
rc=$?; echo "micro rc $rc"; fatal $rc micro
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_exact.py \
  tests/test_gpu_vfilter.py > gpurun_out/r06_t3.log 2>&1
rc=$?; echo "tests rc $rc"; fatal $rc tests; [ $rc -eq 0 ] || exit 3
timeout -k 10 600 python bench.py --config kitti_raw --no-cpu-baseline --pmc off --spread-passes 2 > gpurun_out/r06_bench_kitti_raw_b.json 2> gpurun_out/r06_bench_kitti_raw_b.log
rc=$?; echo "bench raw rc $rc"; fatal $rc raw
