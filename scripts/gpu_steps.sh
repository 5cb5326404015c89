#!/bin/bash
# Run GPU steps in order on the gpurun box; each step has its own time limit.  A step that ends with a
# fault-like status (abort 134, segfault 139, timeout 124/137, or anything other than 0/1/5) stops the
# chain so nothing else touches the GPU after a fault.  Logs go to gpurun_out/<name>.log.
#   scripts/gpu_steps.sh "name:seconds:command args" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
    name="${spec%%:*}"; rest="${spec#*:}"
    secs="${rest%%:*}"; cmd="${rest#*:}"
    echo "[$(date +%T)] start $name ($secs s): $cmd" >> gpurun_out/steps.log
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "[$(date +%T)] end $name rc=$rc" >> gpurun_out/steps.log
    case $rc in
        0|1|5) ;;
        *) echo "stopping after $name (rc=$rc)" >> gpurun_out/steps.log; exit $rc ;;
    esac
done
exit 0
