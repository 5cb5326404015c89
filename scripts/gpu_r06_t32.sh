# kernel trace of the frame loop (e2e): where the per-frame device time goes (voxel filter on pinned input, ICP, map)
cd /root/repo && export TMPDIR=/tmp
mkdir -p /tmp/prof; rm -rf /tmp/prof/e2e
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof/e2e -o run -- python bench.py --config kitti_e2e --no-cpu-baseline > gpurun_out/prof_e2e.json 2> gpurun_out/prof_e2e.log
rc=$?; echo "prof rc $rc"; [ $rc -eq 0 ] || exit 4
db=$(find /tmp/prof/e2e -name '*.db' | head -1)
python scripts/db_kernel_stats.py "$db" > gpurun_out/r06_e2e_kernel_stats.csv
