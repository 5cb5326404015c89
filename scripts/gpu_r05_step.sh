cd /root/repo && export TMPDIR=/tmp
# stop at the first step that faults, aborts or times out (134/139/124/137); test failures continue to the probes
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_exact.py tests/test_gpu_seqsum.py tests/test_gpu_bench_workload.py tests/test_gpu_batch.py tests/test_gpu_devmap.py tests/test_gpu_odometry.py > gpurun_out/t1.log 2>&1
rc=$?; echo "tests rc $rc"; fatal $rc tests
LO_ICP_LIB=lidar_odometry_amd/liblo_icp_diagx.so timeout -k 10 300 python scripts/exact_stamps.py > gpurun_out/st1.log 2>&1
rc=$?; echo "stamps rc $rc"; fatal $rc stamps
rm -f gpurun_out/ph2.log
for L in diag xc1 xc2; do
  echo "== $L" >> gpurun_out/ph2.log
  LO_DIAG_LIB=lidar_odometry_amd/liblo_icp_$L.so timeout -k 10 300 python scripts/pko_exact_phases.py >> gpurun_out/ph2.log 2>&1
  rc=$?; fatal $rc "phases $L"; [ $rc -eq 0 ] || exit 3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof6 -o run -- python bench.py --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --steps 300 --warmup 20 > gpurun_out/b2.log 2>&1
echo "prof rc $?"
