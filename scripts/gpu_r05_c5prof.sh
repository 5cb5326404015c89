cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
rm -rf /tmp/prof/c5; mkdir -p /tmp/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof/c5 -o run -- python bench.py --mode ${1:-exact} --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 12 --steps 100 --warmup 5 > gpurun_out/c5prof.json 2> gpurun_out/c5prof.log
rc=$?; echo "prof rc $rc"; fatal $rc prof
db=$(find /tmp/prof/c5 -name '*.db' | head -1)
python scripts/db_kernel_stats.py "$db" > gpurun_out/r05_c5_db_stats.csv
python scripts/db_kernel_hist.py "$db" "k_correspond(" 8000 > gpurun_out/r05_c5_corr_hist.txt
python scripts/db_kernel_hist.py "$db" "k_pko_t" 10000 >> gpurun_out/r05_c5_corr_hist.txt
python scripts/db_kernel_hist.py "$db" "k_pko_tx" 10000 >> gpurun_out/r05_c5_corr_hist.txt
python scripts/db_kernel_hist.py "$db" "k_exact_scale_c" 0 >> gpurun_out/r05_c5_corr_hist.txt
