# frame loop: the keyframe map update on the map's own stream (the next frame's voxel filter overlaps it); tests + A/B
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; *) echo "rc $1 in $2";; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_odometry.py tests/test_gpu_devmap.py tests/test_gpu_kdtree.py > gpurun_out/t34_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t34_tests.log; fatal $rc tests; [ $rc -eq 0 ] || exit 3
for r in 1 2; do
  for a in 1 0; do
    LO_DM_ASYNC=$a timeout -k 10 300 python bench.py --config kitti_e2e > gpurun_out/t34_e2e_async${a}_$r.json 2> gpurun_out/t34_e2e_async${a}_$r.log; fatal $? e2e$a
  done
done
echo ok
