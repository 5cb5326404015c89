# A/B: the exact candidates' adder with pinned two-stage reads (default) vs the r05 loop (liblo_icp_xcv0.so); exact tests
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_exact.py \
  tests/test_gpu_bench_workload.py > gpurun_out/r06_t13.log 2>&1
rc=$?; echo "tests rc $rc"; fatal $rc tests; [ $rc -eq 0 ] || exit 3
for V in new old new old; do
  if [ $V = old ]; then export LO_ICP_LIB=lidar_odometry_amd/liblo_icp_xcv0.so; else unset LO_ICP_LIB; fi
  timeout -k 10 600 python bench.py --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 --spread-passes 2 > gpurun_out/r06_xc_$V.json 2> gpurun_out/r06_xc_$V.log
  rc=$?; echo "bench $V rc $rc"; fatal $rc bench
  python3 -c "import json;d=json.loads(open('gpurun_out/r06_xc_$V.json').read().strip().splitlines()[-1]);print('$V', d['value'], d['value_spread']['median'], d['other_mode']['value'])"
done
unset LO_ICP_LIB
LO_DIAG_LIB=lidar_odometry_amd/liblo_icp_diags.so timeout -k 10 300 python scripts/pko_exact_phases.py kitti > gpurun_out/r06_pko_exact_phases_b.txt 2>&1
rc=$?; echo "phases rc $rc"; fatal $rc phases
