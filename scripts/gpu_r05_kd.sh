cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_odometry.py tests/test_gpu_devmap.py tests/test_gpu_kdtree.py > gpurun_out/t4.log 2>&1
rc=$?; echo "tests rc $rc"; fatal $rc tests; [ $rc -eq 0 ] || exit 3
timeout -k 10 600 python bench.py --config kitti_e2e_kdtree --no-cpu-baseline --steps 120 > gpurun_out/e2e_kd.json 2> gpurun_out/e2e_kd.log
echo "e2e kd rc $?"
bash scripts/gpu_r05_c5prof.sh exact
