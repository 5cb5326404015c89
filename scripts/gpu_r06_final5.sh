# round 6, last check of the committed tree: the whole GPU suite and smoke()
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r06_gpu_tests_final.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/r06_gpu_tests_final.log; fatal $rc tests; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke_final.log 2>&1
rc=$?; echo "smoke rc $rc"; fatal $rc smoke
