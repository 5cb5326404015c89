# Round 6: filter in one workgroup + bucket-sorted big voxels (tests, raw + e2e benches), the solve's cold latency
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 60 scripts/solve_microbench > gpurun_out/r06_solve_microbench.txt 2>&1
rc=$?; echo "micro rc $rc"; fatal $rc micro
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_vfilter.py \
  tests/test_gpu_odometry.py tests/test_gpu_exact.py -k "raw or vfilter or voxel or odometry or frame or flush or overflow" > gpurun_out/r06_t4.log 2>&1
rc=$?; echo "tests rc $rc"; fatal $rc tests; [ $rc -eq 0 ] || exit 3
timeout -k 10 600 python bench.py --config kitti_raw --no-cpu-baseline --pmc off --spread-passes 2 > gpurun_out/r06_bench_kitti_raw_c.json 2> gpurun_out/r06_bench_kitti_raw_c.log
rc=$?; echo "bench raw rc $rc"; fatal $rc raw
timeout -k 10 600 python bench.py --config kitti_e2e --no-cpu-baseline --pmc off > gpurun_out/r06_bench_kitti_e2e_c.json 2> gpurun_out/r06_bench_kitti_e2e_c.log
rc=$?; echo "bench e2e rc $rc"; fatal $rc e2e
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_map_patch.py > gpurun_out/r06_t4b.log 2>&1
rc=$?; echo "map tests rc $rc"; fatal $rc maptests
timeout -k 10 600 python scripts/map_sync_timing.py 300 > gpurun_out/r06_map_sync_timing.txt 2>&1
rc=$?; echo "map timing rc $rc"; fatal $rc maptiming
