# Round 6: exact candidates start at launch, adder lanes masked, glibc sinf in the solve: exact tests, the PKO timeline,
# KITTI exact bench (short), map sync timing.  Stops at a fault, abort or time limit.
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_exact.py \
  tests/test_gpu_bench_workload.py tests/test_gpu_pipeline.py tests/test_gpu_map_patch.py > gpurun_out/r06_t7.log 2>&1
rc=$?; echo "tests rc $rc"; fatal $rc tests; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python scripts/pko_exact_timeline.py kitti > gpurun_out/r06_pko_timeline_c.txt 2>&1
rc=$?; echo "timeline rc $rc"; fatal $rc timeline
timeout -k 10 600 python bench.py --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 --spread-passes 3 > gpurun_out/r06_bench_kitti_f.json 2> gpurun_out/r06_bench_kitti_f.log
rc=$?; echo "bench rc $rc"; fatal $rc bench
timeout -k 10 600 python scripts/map_sync_timing.py 300 > gpurun_out/r06_map_sync_timing.txt 2>&1
rc=$?; echo "map timing rc $rc"; fatal $rc maptiming
