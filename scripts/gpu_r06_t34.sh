# A/B: the exact candidates' adder wave (and its solving lane) at issue priority 3 (liblo_icp_prio.so, -DLO_XC_PRIO)
# against the product build, same box, alternating, two rounds
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
for L in base prio base prio; do
  if [ $L = prio ]; then export LO_ICP_LIB=lidar_odometry_amd/liblo_icp_prio.so; else export LO_ICP_LIB=lidar_odometry_amd/liblo_icp.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 --spread-passes 2 > gpurun_out/t34_$L.json 2> gpurun_out/t34_$L.log
  rc=$?; echo "bench $L rc $rc"; fatal $rc bench
  python3 -c "import json;d=json.loads(open('gpurun_out/t34_$L.json').read().strip().splitlines()[-1]);print('$L', d['value'], d['value_spread']['median'], d['other_mode']['value'])"
done
