# Factored long sums (k_exact_terms writes 14 factor rows; the column sums form the products) against the 43 stored
# columns (liblo_icp_nf.so, LO_EXACT_FACTORED=0), both with 16-B run loads: parity tests on each, then the C5 rate
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
for L in icp icp_nf; do
  LO_ICP_LIB=lidar_odometry_amd/liblo_$L.so timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_seqsum.py tests/test_gpu_exact.py tests/test_gpu_bench_workload.py > gpurun_out/fac_t_$L.log 2>&1
  rc=$?; echo "tests $L rc $rc"; fatal $rc "tests $L"; [ $rc -eq 0 ] || exit 3
done
bash scripts/gpu_r05_walkab.sh
