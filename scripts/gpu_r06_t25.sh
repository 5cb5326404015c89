# EM loop in buffer-half pairs: PKO parity + exact tests, KITTI bench (live EM cycles)
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; *) echo "rc $1 in $2";; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_exact.py tests/test_gpu_batch.py > gpurun_out/t25_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t25_tests.log; fatal $rc tests; [ $rc -eq 0 ] || exit 3
timeout -k 10 600 python bench.py --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 > gpurun_out/t25_kitti.json 2> gpurun_out/t25_kitti.log; fatal $? kitti
echo ok
