# Round 6: which part bounds the exact PKO launch (diag stamps), the raw-scan exact kernel trace, and the C5 leg's
# trace (the primary roofline timing reproduced from rocprofv3).  Stops at a fault, abort or time limit.
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
mkdir -p /tmp/prof
timeout -k 10 300 python scripts/pko_exact_timeline.py kitti > gpurun_out/r06_pko_timeline.txt 2>&1
rc=$?; echo "timeline rc $rc"; fatal $rc timeline
rm -rf /tmp/prof/raw
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof/raw -o run -- python bench.py --config kitti_raw --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 --steps 200 --warmup 5 --spread-passes 0 > gpurun_out/prof_raw.json 2> gpurun_out/prof_raw.log
rc=$?; echo "prof raw rc $rc"; fatal $rc prof_raw
db=$(find /tmp/prof/raw -name '*.db' | head -1)
python scripts/db_kernel_stats.py "$db" > gpurun_out/r06_raw_exact_kernel_stats.csv
rm -rf /tmp/prof/c5
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof/c5 -o run -- python bench.py --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 12 --steps 100 --warmup 5 --spread-passes 0 > gpurun_out/c5prof.json 2> gpurun_out/c5prof.log
rc=$?; echo "prof c5 rc $rc"; fatal $rc prof_c5
db=$(find /tmp/prof/c5 -name '*.db' | head -1)
python scripts/c5_trace_rr.py "$db" gpurun_out/c5prof.json --out gpurun_out/r06_1m_trace_summary.json > /dev/null
python scripts/db_kernel_stats.py "$db" > gpurun_out/r06_c5_db_stats.csv
