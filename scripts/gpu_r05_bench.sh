cd /root/repo && export TMPDIR=/tmp
timeout -k 10 1000 python bench.py > gpurun_out/r05_bench_kitti.json 2> gpurun_out/r05_bench_kitti.log
echo "bench rc $?"
