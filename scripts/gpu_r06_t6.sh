# Round 6: filter without the last-block hand-off, the wide device-count scale inside k_exact_scale_cd (tests, raw
# kernel trace, raw / e2e benches).  Stops at a fault, abort or time limit.
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_exact.py \
  tests/test_gpu_vfilter.py tests/test_gpu_odometry.py > gpurun_out/r06_t6.log 2>&1
rc=$?; echo "tests rc $rc"; fatal $rc tests; [ $rc -eq 0 ] || exit 3
mkdir -p /tmp/prof; rm -rf /tmp/prof/raw
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof/raw -o run -- python bench.py --config kitti_raw --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 --steps 200 --warmup 5 --spread-passes 0 > gpurun_out/prof_raw.json 2> gpurun_out/prof_raw.log
rc=$?; echo "prof raw rc $rc"; fatal $rc prof_raw
db=$(find /tmp/prof/raw -name '*.db' | head -1)
python scripts/db_kernel_stats.py "$db" > gpurun_out/r06_raw_exact_kernel_stats_c.csv
timeout -k 10 600 python bench.py --config kitti_raw --no-cpu-baseline --pmc off --spread-passes 2 > gpurun_out/r06_bench_kitti_raw_e.json 2> gpurun_out/r06_bench_kitti_raw_e.log
rc=$?; echo "bench raw rc $rc"; fatal $rc raw
timeout -k 10 600 python bench.py --config kitti_e2e --no-cpu-baseline --pmc off > gpurun_out/r06_bench_kitti_e2e_e.json 2> gpurun_out/r06_bench_kitti_e2e_e.log
rc=$?; echo "bench e2e rc $rc"; fatal $rc e2e
