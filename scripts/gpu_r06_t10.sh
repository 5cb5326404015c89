cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
LO_DIAG_LIB=lidar_odometry_amd/liblo_icp_diags.so timeout -k 10 300 python scripts/pko_exact_phases.py kitti > gpurun_out/r06_pko_exact_phases.txt 2>&1
rc=$?; echo "phases rc $rc"; fatal $rc phases
