# KDTree / loop-closure with PKO candidates (k_pick_knn), wave-per-query brute force, adaptive loop grid
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; *) echo "rc $1 in $2";; esac; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kdtree.py tests/test_gpu_loop.py tests/test_gpu_exact.py > gpurun_out/t15_tests.log 2>&1
rc=$?; tail -5 gpurun_out/t15_tests.log; fatal $rc tests; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python scripts/loop_diag.py exact > gpurun_out/t15_loopdiag.txt 2>&1; fatal $? diag
timeout -k 10 300 python bench.py --config kitti_loop --mode exact --steps 300 --warmup 20 > gpurun_out/t15_loop_exact.json 2> gpurun_out/t15_loop_exact.log; fatal $? loopx
timeout -k 10 300 python bench.py --config kitti_loop --mode fast --no-cpu-baseline --steps 300 --warmup 20 > gpurun_out/t15_loop_fast.json 2> gpurun_out/t15_loop_fast.log; fatal $? loopf
timeout -k 10 300 python bench.py --config kitti_kdtree --mode exact --no-cpu-baseline --pmc off --steps 200 --warmup 5 --spread-passes 0 > gpurun_out/t15_kd_exact.json 2> gpurun_out/t15_kd_exact.log; fatal $? kdx
timeout -k 10 300 python bench.py --config kitti_kdtree --no-cpu-baseline --pmc off --steps 200 --warmup 5 --spread-passes 0 > gpurun_out/t15_kd_fast.json 2> gpurun_out/t15_kd_fast.log; fatal $? kdf
echo ok
