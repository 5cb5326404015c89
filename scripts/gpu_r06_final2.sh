# round 6: the remaining bench configurations and the kernel statistics of the exact KITTI / 1M / loop steps
cd /root/repo && export TMPDIR=/tmp
bash scripts/gpu_r06_allbench.sh patch1m kitti_raw kitti_kdtree kitti_e2e kitti_loop || exit 4
bash scripts/gpu_r06_prof.sh kitti exact 300 || exit 4
