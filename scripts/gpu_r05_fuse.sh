# Fused long-column classification (one launch: chunk sums + drift + classification with a look-back) vs the
# three-launch path (LO_MW_SPLIT=1): parity tests, then the 1M-point exact rate of each, then the fused profile
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_seqsum.py tests/test_gpu_exact.py tests/test_gpu_bench_workload.py > gpurun_out/t8.log 2>&1
rc=$?; echo "tests rc $rc"; fatal $rc tests; [ $rc -eq 0 ] || exit 3
for V in fused split; do
  if [ $V = split ]; then export LO_MW_SPLIT=1; fi
  timeout -k 10 400 python bench.py --config patch1m --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --steps 40 --warmup 4 > gpurun_out/fuse_b_$V.json 2> gpurun_out/fuse_b_$V.log
  rc=$?; echo "$V rc $rc"; fatal $rc "bench $V"
done
unset LO_MW_SPLIT
bash scripts/gpu_r05_prof.sh patch1m exact 40
