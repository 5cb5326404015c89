# every bench configuration with its defaults, one JSON line each into gpurun_out/r06_bench_<config>.json; stops at
# a fault, abort or time limit
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
for C in "$@"; do
  timeout -k 10 900 python bench.py --config $C > gpurun_out/r06_bench_$C.json 2> gpurun_out/r06_bench_$C.log
  rc=$?; echo "bench $C rc $rc"; fatal $rc $C
done
