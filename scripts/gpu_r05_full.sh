# The whole GPU suite, then the C2 (KITTI-like) and C5 (1M-point) exact rates
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/tfull.log 2>&1
rc=$?; echo "tests rc $rc"; fatal $rc tests; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --config kitti --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --steps 2000 --warmup 50 > gpurun_out/full_kitti.json 2> gpurun_out/full_kitti.log
rc=$?; echo "kitti rc $rc"; fatal $rc kitti
timeout -k 10 300 python bench.py --config patch1m --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --steps 40 --warmup 4 > gpurun_out/full_c5.json 2> gpurun_out/full_c5.log
rc=$?; echo "c5 rc $rc"; fatal $rc c5
