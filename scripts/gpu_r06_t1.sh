# Round 6, first GPU pass: the changed GPU tests (count-aware exact scale, batch attribute, map flush, C4 bench
# workload), then the raw-scan and KITTI bench lines.  Stops at a fault, abort or time limit.
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_exact.py tests/test_gpu_vfilter.py tests/test_gpu_odometry.py tests/test_gpu_batch.py \
  tests/test_gpu_bench_workload.py > gpurun_out/r06_t1.log 2>&1
rc=$?; echo "tests rc $rc"; fatal $rc tests
timeout -k 10 600 python bench.py --config kitti_raw > gpurun_out/r06_bench_kitti_raw.json 2> gpurun_out/r06_bench_kitti_raw.log
rc=$?; echo "bench raw rc $rc"; fatal $rc raw
timeout -k 10 900 python bench.py > gpurun_out/r06_bench_kitti.json 2> gpurun_out/r06_bench_kitti.log
rc=$?; echo "bench kitti rc $rc"; fatal $rc kitti
