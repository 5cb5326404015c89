# grid kNN: lane-minimum first pass for unseeded searches; k_knn_brute without scratch (visit-order ranking of the
# tie set by one lane); KDTree / loop / odometry tests, KDTree bench + kernel stats
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; *) echo "rc $1 in $2";; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kdtree.py tests/test_gpu_loop.py tests/test_gpu_odometry.py tests/test_gpu_bench_workload.py > gpurun_out/t27_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t27_tests.log; fatal $rc tests; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --config kitti_kdtree --pmc off --steps 300 --warmup 10 --spread-passes 0 > gpurun_out/t27_kd.json 2> gpurun_out/t27_kd.log; fatal $? kd
bash scripts/gpu_r06_prof.sh kitti_kdtree exact 300 || exit 4
echo ok
