#!/bin/bash
# Host-side helper: run one gpurun command, waiting and trying again only while the pool reports no box / a
# transient infrastructure event (nothing ran).  A command that ran -- whatever its exit code -- is never repeated.
#   scripts/gpu_retry.sh <timeout-s> '<command>'
T="$1"; shift
for i in 1 2 3 4 5 6 7 8 9 10; do
    out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
    if echo "$out" | grep -q "status=transient\|backing off"; then
        echo "[gpu_retry] attempt $i: $(echo "$out" | grep -o 'status=transient.*\|retry in [0-9]*s' | head -1)" >&2
        w=$(echo "$out" | grep -o 'retry in [0-9]*s' | grep -o '[0-9]*' | head -1)
        sleep $(( ${w:-90} + 20 ))
        continue
    fi
    echo "$out"
    exit 0
done
echo "[gpu_retry] gave up" >&2
exit 3
