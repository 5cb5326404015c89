# Same-box A/B: classification heads kept in registers (0 / 1 / 2 / 3 per thread; 0 = the record pass always runs),
# after the parity tests of the long-column sums on each variant
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
for L in rh1 rh2 rh3; do
  LO_ICP_LIB=lidar_odometry_amd/liblo_icp_$L.so timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_seqsum.py tests/test_gpu_bench_workload.py > gpurun_out/rh_t_$L.log 2>&1
  rc=$?; echo "tests $L rc $rc"; fatal $rc "tests $L"; [ $rc -eq 0 ] || exit 3
done
for r in 1 2; do
for L in rh0 rh1 rh2 rh3; do
  LO_ICP_LIB=lidar_odometry_amd/liblo_icp_$L.so timeout -k 10 300 python bench.py --config patch1m --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --steps 40 --warmup 4 > gpurun_out/rhab_${L}_$r.json 2> gpurun_out/rhab_${L}_$r.log
  rc=$?; echo "$L $r rc $rc"; fatal $rc "bench $L"
done
done
