cd /root/repo && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_exact.py tests/test_gpu_seqsum.py tests/test_gpu_bench_workload.py > gpurun_out/t1.log 2>&1
echo "tests rc $?"
LO_ICP_LIB=lidar_odometry_amd/liblo_icp_diagx.so timeout -k 10 300 python scripts/exact_stamps.py > gpurun_out/st1.log 2>&1
echo "stamps rc $?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run -- python bench.py --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --steps 300 --warmup 20 > gpurun_out/b2.log 2>&1
echo "prof rc $?"
LO_DIAG_LIB=lidar_odometry_amd/liblo_icp_diag.so timeout -k 10 300 python scripts/pko_exact_phases.py > gpurun_out/ph1.log 2>&1
echo "phases rc $?"
