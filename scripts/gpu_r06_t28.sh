# exact scale widths 3 / 5 / 6: exact + batch + bench-workload tests, KITTI and MID360 lines, KITTI exact kernel stats
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; *) echo "rc $1 in $2";; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_exact.py tests/test_gpu_batch.py tests/test_gpu_bench_workload.py > gpurun_out/t28_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t28_tests.log; fatal $rc tests; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 > gpurun_out/t28_kitti.json 2> gpurun_out/t28_kitti.log; fatal $? kitti
timeout -k 10 300 python bench.py --config mid360 --no-cpu-baseline --pmc off --batch "" --sequences 0 > gpurun_out/t28_mid.json 2> gpurun_out/t28_mid.log; fatal $? mid
bash scripts/gpu_r06_prof.sh kitti exact 300 || exit 4
echo ok
