# Parity tests of the long-column sums, the walk's cycle split (liblo_icp_diagx.so) and the 1M-point exact rate
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_seqsum.py tests/test_gpu_exact.py tests/test_gpu_bench_workload.py > gpurun_out/t9.log 2>&1
rc=$?; echo "tests rc $rc"; fatal $rc tests; [ $rc -eq 0 ] || exit 3
LO_ICP_LIB=lidar_odometry_amd/liblo_icp_diagx.so timeout -k 10 400 python scripts/exact_stamps.py --config patch1m > gpurun_out/walk_st.log 2>&1
rc=$?; echo "stamps rc $rc"; fatal $rc stamps
timeout -k 10 400 python bench.py --config patch1m --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --steps 40 --warmup 4 > gpurun_out/walk_b.json 2> gpurun_out/walk_b.log
rc=$?; echo "bench rc $rc"; fatal $rc bench
