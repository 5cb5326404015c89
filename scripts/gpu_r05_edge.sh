# A/B of the long-column edge margin (kMwEdgeBits 9 / 10 / 11, all with the exact stamps): walk statistics and the
# 1M-point exact rate; results are bitwise the same by construction (the walk's checks)
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
for L in diagx edge10 edge11; do
  LO_ICP_LIB=lidar_odometry_amd/liblo_icp_$L.so timeout -k 10 400 python scripts/exact_stamps.py --config patch1m > gpurun_out/edge_st_$L.log 2>&1
  rc=$?; fatal $rc "stamps $L"
  LO_ICP_LIB=lidar_odometry_amd/liblo_icp_$L.so timeout -k 10 400 python bench.py --config patch1m --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --steps 40 --warmup 4 > gpurun_out/edge_b_$L.json 2> gpurun_out/edge_b_$L.log
  rc=$?; echo "$L rc $rc"; fatal $rc "bench $L"
done
LO_ICP_LIB=lidar_odometry_amd/liblo_icp_edge11.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_seqsum.py tests/test_gpu_bench_workload.py > gpurun_out/t7.log 2>&1
echo "tests edge11 rc $?"
