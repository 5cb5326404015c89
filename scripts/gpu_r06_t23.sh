# loop ICP with pinned curr upload; kdtree tests; loop + kdtree benches
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; *) echo "rc $1 in $2";; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_loop.py tests/test_gpu_kdtree.py > gpurun_out/t23_tests.log 2>&1
rc=$?; tail -2 gpurun_out/t23_tests.log; fatal $rc tests; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --config kitti_loop --mode exact --steps 400 --warmup 20 > gpurun_out/t23_loop_exact.json 2> gpurun_out/t23_loop_exact.log; fatal $? loopx
timeout -k 10 300 python bench.py --config kitti_loop --mode fast --steps 400 --warmup 20 > gpurun_out/t23_loop_fast.json 2> gpurun_out/t23_loop_fast.log; fatal $? loopf
timeout -k 10 300 python bench.py --config kitti_kdtree --mode exact --pmc off --steps 200 --warmup 5 --spread-passes 0 > gpurun_out/t23_kd_exact.json 2> gpurun_out/t23_kd_exact.log; fatal $? kdx
echo ok
