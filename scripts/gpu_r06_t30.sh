# A/B: the exact candidates' consumer with the next group's packed products between the adds (liblo_icp.so) against
# the read-ahead loop (liblo_icp_ab0.so, HEAD's lo_pko_body.h), exact parity tests, and the PKO timeline of the new build
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_exact.py tests/test_gpu_bench_workload.py > gpurun_out/t30_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t30_tests.log; fatal $rc tests; [ $rc -eq 0 ] || exit 5
for L in ab0 new ab0 new; do
  if [ $L = new ]; then export LO_ICP_LIB=lidar_odometry_amd/liblo_icp.so; else export LO_ICP_LIB=lidar_odometry_amd/liblo_icp_ab0.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 --spread-passes 2 > gpurun_out/t30_$L.json 2> gpurun_out/t30_$L.log
  rc=$?; echo "bench $L rc $rc"; fatal $rc bench
  python3 -c "import json;d=json.loads(open('gpurun_out/t30_$L.json').read().strip().splitlines()[-1]);print('$L', d['value'], d['value_spread']['median'], d['other_mode']['value'], d.get('cpu_baseline',{}) and d['cpu_baseline'].get('parity'))"
done
unset LO_ICP_LIB
timeout -k 10 300 python scripts/pko_exact_timeline.py kitti > gpurun_out/t30_timeline.txt 2>&1
rc=$?; echo "timeline rc $rc"; fatal $rc timeline; head -12 gpurun_out/t30_timeline.txt
