# loop-closure ICP: batched LDS staging of the all-pairs kernels; bench + kernel trace
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; *) echo "rc $1 in $2";; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_loop.py > gpurun_out/t21_tests.log 2>&1
rc=$?; tail -2 gpurun_out/t21_tests.log; fatal $rc tests; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --config kitti_loop --mode exact --steps 300 --warmup 20 > gpurun_out/t21_loop_exact.json 2> gpurun_out/t21_loop_exact.log; fatal $? loopx
mkdir -p /tmp/prof; rm -rf /tmp/prof/loop
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof/loop -o run -- python bench.py --config kitti_loop --mode exact --no-cpu-baseline --steps 300 --warmup 10 > gpurun_out/prof_loop7.json 2> gpurun_out/prof_loop7.log
rc=$?; echo "prof loop rc $rc"; fatal $rc prof
db=$(find /tmp/prof/loop -name '*.db' | head -1)
python scripts/db_kernel_stats.py "$db" > gpurun_out/r06_loop_exact_kernel_stats7.csv
python scripts/kernel_gaps.py "$db" > gpurun_out/r06_loop_gaps7.txt 2>&1
echo ok
