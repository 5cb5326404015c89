cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
for PM in 1 2 3; do
  LO_PIPE_MAIN=$PM timeout -k 10 300 python bench.py --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 --steps 2000 --warmup 40 > gpurun_out/pipe_$PM.json 2> gpurun_out/pipe_$PM.log
  rc=$?; echo "pipe $PM rc $rc"; fatal $rc pipe
done
