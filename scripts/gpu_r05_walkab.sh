# Same-box A/B of the long-column walk: the current one (LDS-recorded chain, chain again after a failure) against the
# previous one (liblo_icp_wold.so, built from the previous commit's walk), 1M-point exact rate, three rounds alternating
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
for r in 1 2; do
for L in icp icp_nf; do
  LO_ICP_LIB=lidar_odometry_amd/liblo_$L.so timeout -k 10 300 python bench.py --config patch1m --mode exact --no-cpu-baseline --pmc off --batch "" --sequences 0 --steps 40 --warmup 4 > gpurun_out/wab_${L}_$r.json 2> gpurun_out/wab_${L}_$r.log
  rc=$?; echo "$L $r rc $rc"; fatal $rc "bench $L"
done
done
