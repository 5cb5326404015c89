# A/B: the PKO launch with and without its EM chain (liblo_icp_diag.so vs liblo_icp_xc3.so, both with the PKO stamps):
# GN iterations per second in both arithmetic modes -- the upper bound of what hiding the EM could buy
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
for LIB in diag xc3; do
  for M in exact fast; do
    LO_ICP_LIB=lidar_odometry_amd/liblo_icp_$LIB.so timeout -k 10 300 python bench.py --mode $M --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 --steps 1000 --warmup 40 > gpurun_out/ab_em_${LIB}_$M.json 2> gpurun_out/ab_em_${LIB}_$M.log
    rc=$?; echo "ab $LIB $M rc $rc"; fatal $rc ab
  done
done
