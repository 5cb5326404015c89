# rocprofv3 kernel statistics of one bench configuration's timed steps: gpurun_out/r06_<config>_<mode>_kernel_stats.csv
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
mkdir -p /tmp/prof
C=${1:-kitti}
M=${2:-exact}
rm -rf /tmp/prof/$C$M
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof/$C$M -o run -- python bench.py --config $C --mode $M --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 --spread-passes 0 --steps ${3:-200} --warmup 5 > gpurun_out/prof_$C$M.json 2> gpurun_out/prof_$C$M.log
rc=$?; echo "prof rc $rc"; fatal $rc prof
db=$(find /tmp/prof/$C$M -name '*.db' | head -1)
python scripts/db_kernel_stats.py "$db" > gpurun_out/r06_${C}_${M}_kernel_stats.csv
