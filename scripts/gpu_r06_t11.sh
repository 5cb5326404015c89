cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
timeout -k 10 60 scripts/chain_microbench > gpurun_out/r06_chain_microbench.txt 2>&1
rc=$?; echo "chain rc $rc"; fatal $rc chain
timeout -k 10 60 scripts/consumer_microbench > gpurun_out/r06_consumer_microbench.txt 2>&1
rc=$?; echo "consumer rc $rc"; fatal $rc consumer
