# A/B: one PKO workgroup per CU (LO_PKO_SOLO=1) in the exact KITTI bench, and its PKO timeline
cd /root/repo && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc $1 in $2"; exit 4;; esac; }
for S in 0 1 0 1; do
  LO_PKO_SOLO=$S timeout -k 10 600 python bench.py --no-cpu-baseline --pmc off --batch "" --sequences 0 --c5 0 --spread-passes 2 > gpurun_out/r06_solo$S.json 2> gpurun_out/r06_solo$S.log
  rc=$?; echo "bench solo=$S rc $rc"; fatal $rc bench
  python3 -c "import json;d=json.loads(open('gpurun_out/r06_solo$S.json').read().strip().splitlines()[-1]);print('solo=$S', d['value'], d['value_spread']['median'], d['other_mode']['value'])"
done
LO_PKO_SOLO=1 timeout -k 10 300 python scripts/pko_exact_timeline.py kitti > gpurun_out/r06_pko_timeline_solo.txt 2>&1
rc=$?; echo "timeline rc $rc"; fatal $rc timeline
