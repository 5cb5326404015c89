# device-count scale widths 3 / 5 / 6: exact + vfilter + odometry tests, raw and e2e lines
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; *) echo "rc $1 in $2";; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_exact.py tests/test_gpu_vfilter.py tests/test_gpu_odometry.py > gpurun_out/t29_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t29_tests.log; fatal $rc tests; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --config kitti_raw --no-cpu-baseline --pmc off --batch "" --sequences 0 > gpurun_out/t29_raw.json 2> gpurun_out/t29_raw.log; fatal $? raw
timeout -k 10 300 python bench.py --config kitti_e2e --no-cpu-baseline > gpurun_out/t29_e2e.json 2> gpurun_out/t29_e2e.log; fatal $? e2e
echo ok
