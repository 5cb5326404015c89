# End of round 5: the whole GPU suite, the C5 bench line and its kernel stats, the walk's cycle split, smoke()
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/tfinal.log 2>&1
rc=$?; echo "tests rc $rc"; fatal $rc tests; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc $rc"; fatal $rc smoke; [ $rc -eq 0 ] || exit 3
bash scripts/gpu_r05_allbench.sh patch1m || exit 4
bash scripts/gpu_r05_prof.sh patch1m exact 40 || exit 4
LO_ICP_LIB=lidar_odometry_amd/liblo_icp_diagx.so timeout -k 10 400 python scripts/exact_stamps.py --config patch1m > gpurun_out/walk_st.log 2>&1
rc=$?; echo "stamps rc $rc"; fatal $rc stamps
