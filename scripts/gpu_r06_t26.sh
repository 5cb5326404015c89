# in-launch candidate abort again, now that the EM is ~1076 cycles per iteration: tests + same-box A/B
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; *) echo "rc $1 in $2";; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_exact.py tests/test_gpu_pipeline.py tests/test_gpu_kdtree.py tests/test_gpu_bench_workload.py > gpurun_out/t26_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t26_tests.log; fatal $rc tests; [ $rc -eq 0 ] || exit 3
for r in 1 2; do
  for a in 1 0; do
    LO_CAND_ABORT=$a timeout -k 10 300 python bench.py --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 > gpurun_out/t26_abort${a}_$r.json 2> gpurun_out/t26_abort${a}_$r.log; fatal $? ab$a
  done
done
echo ok
