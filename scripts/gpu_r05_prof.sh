cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
mkdir -p /tmp/prof
for M in exact fast; do
  rm -rf /tmp/prof/$M
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof/$M -o run -- python bench.py --mode $M --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 --steps 400 --warmup 20 > gpurun_out/prof_$M.json 2> gpurun_out/prof_$M.log
  rc=$?; echo "prof $M rc $rc"; fatal $rc prof
  f=$(find /tmp/prof/$M -name '*kernel_stats.csv' | head -1)
  grep -E '"Name"|lo::' "$f" > gpurun_out/r05_kitti_${M}_kernel_stats.csv
  db=$(find /tmp/prof/$M -name '*.db' | head -1)
  [ -n "$db" ] && python scripts/db_kernel_stats.py "$db" > gpurun_out/r05_kitti_${M}_db_stats.csv
done
ls -la /tmp/prof/*
