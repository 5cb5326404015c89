# round 6: kernel statistics of the exact 1M-point, KDTree and raw-scan steps
cd /root/repo && export TMPDIR=/tmp
bash scripts/gpu_r06_prof.sh patch1m exact 40 || exit 4
bash scripts/gpu_r06_prof.sh kitti_kdtree exact 300 || exit 4
bash scripts/gpu_r06_prof.sh kitti_raw exact 300 || exit 4
