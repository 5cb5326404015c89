# kernel traces of the exact loop-closure ICP and the exact KDTree step (C4)
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
mkdir -p /tmp/prof; rm -rf /tmp/prof/loop /tmp/prof/kd
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof/loop -o run -- python bench.py --config kitti_loop --mode exact --no-cpu-baseline --pmc off --steps 200 --warmup 10 > gpurun_out/prof_loop.json 2> gpurun_out/prof_loop.log
rc=$?; echo "prof loop rc $rc"; fatal $rc loop
db=$(find /tmp/prof/loop -name '*.db' | head -1)
python scripts/db_kernel_stats.py "$db" > gpurun_out/r06_loop_exact_kernel_stats.csv
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof/kd -o run -- python bench.py --config kitti_kdtree --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 --steps 200 --warmup 5 --spread-passes 0 > gpurun_out/prof_kd.json 2> gpurun_out/prof_kd.log
rc=$?; echo "prof kd rc $rc"; fatal $rc kd
db=$(find /tmp/prof/kd -name '*.db' | head -1)
python scripts/db_kernel_stats.py "$db" > gpurun_out/r06_kd_exact_kernel_stats.csv
