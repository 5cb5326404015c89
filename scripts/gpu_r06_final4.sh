# round 6 (after the EM, scale-width and kNN changes): the loop-closure line's kernel trace and timeline
cd /root/repo && export TMPDIR=/tmp
mkdir -p /tmp/prof; rm -rf /tmp/prof/loop
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof/loop -o run -- python bench.py --config kitti_loop --mode exact --no-cpu-baseline --steps 300 --warmup 10 > gpurun_out/prof_loop_final.json 2> gpurun_out/prof_loop_final.log
rc=$?; echo "prof loop rc $rc"; [ $rc -eq 0 ] || exit 4
db=$(find /tmp/prof/loop -name '*.db' | head -1)
python scripts/db_kernel_stats.py "$db" > gpurun_out/r06_loop_exact_kernel_stats_final.csv
python scripts/kernel_gaps.py "$db" > gpurun_out/r06_loop_timeline_final.txt 2>&1
