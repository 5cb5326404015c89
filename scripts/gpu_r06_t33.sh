# round 6: the KDTree frame loop line, and the 2-rank gloo rehearsal on one GPU (scan-parallel replicas + gather)
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }


timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --check-records --steps 300 --warmup 20 --batch "" --sequences 0 --c5 0 > gpurun_out/r06_bench_kitti_2rank_gloo_1gpu.json 2> gpurun_out/r06_bench_kitti_2rank_gloo_1gpu.log
rc=$?; echo "2rank rc $rc"; fatal $rc 2rank
