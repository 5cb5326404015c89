cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 300 python scripts/pko_exact_timeline.py kitti > gpurun_out/r06_pko_timeline_d.txt 2>&1
rc=$?; echo "timeline rc $rc"; fatal $rc timeline
