# kernel trace of the exact loop-closure ICP after k_pick_knn / k_knn_brute_w / adaptive grid
cd /root/repo && export TMPDIR=/tmp
mkdir -p /tmp/prof; rm -rf /tmp/prof/loop
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof/loop -o run -- python bench.py --config kitti_loop --mode exact --no-cpu-baseline --steps 300 --warmup 10 > gpurun_out/prof_loop2.json 2> gpurun_out/prof_loop2.log
rc=$?; echo "prof loop rc $rc"; [ $rc -eq 0 ] || exit 4
db=$(find /tmp/prof/loop -name '*.db' | head -1)
python scripts/db_kernel_stats.py "$db" > gpurun_out/r06_loop_exact_kernel_stats2.csv
python scripts/kernel_gaps.py "$db" > gpurun_out/r06_loop_gaps.txt 2>&1 || true
