# Round 6: in-launch JS argmin + stopping the exact candidates that were not chosen: exact tests, A/B bench, timeline
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_exact.py \
  tests/test_gpu_bench_workload.py tests/test_gpu_pipeline.py tests/test_gpu_odometry.py tests/test_gpu_vfilter.py > gpurun_out/r06_t12.log 2>&1
rc=$?; echo "tests rc $rc"; fatal $rc tests; [ $rc -eq 0 ] || exit 3
for A in 1 0 1 0; do
  LO_CAND_ABORT=$A timeout -k 10 600 python bench.py --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 --spread-passes 2 > gpurun_out/r06_abort$A.json 2> gpurun_out/r06_abort$A.log
  rc=$?; echo "bench abort=$A rc $rc"; fatal $rc bench
  python3 -c "import json;d=json.loads(open('gpurun_out/r06_abort$A.json').read().strip().splitlines()[-1]);print('abort=$A', d['value'], d['value_spread']['median'], d['other_mode']['value'], d['cpu_baseline'] if 'cpu_baseline' in d else '')"
done
timeout -k 10 300 python scripts/pko_exact_timeline.py kitti > gpurun_out/r06_pko_timeline_e.txt 2>&1
rc=$?; echo "timeline rc $rc"; fatal $rc timeline
