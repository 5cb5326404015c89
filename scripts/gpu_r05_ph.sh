cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_exact.py tests/test_gpu_batch.py tests/test_gpu_bench_workload.py > gpurun_out/t2.log 2>&1
rc=$?; echo "tests rc $rc"; fatal $rc tests; [ $rc -eq 0 ] || exit 3
rm -f gpurun_out/ph3.log
LO_DIAG_LIB=lidar_odometry_amd/liblo_icp_diag.so timeout -k 10 300 python scripts/pko_exact_phases.py >> gpurun_out/ph3.log 2>&1
rc=$?; fatal $rc "phases"
timeout -k 10 300 python bench.py --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 --steps 1000 --warmup 40 > gpurun_out/b3.json 2> gpurun_out/b3.log
echo "bench rc $?"
