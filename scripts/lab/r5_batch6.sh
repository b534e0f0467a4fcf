#!/bin/bash
# round 5, GPU batch 6: the driver's 20 / 5 command vs 200 / 20 -- host clock vs device events, and
# the multi-step graph group size at 20 timed steps
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b6
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[batch] $name: $*" >&2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "[batch] $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then echo "[batch] stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
step build 600 python -c "from sparse_coding__amd.ops import build as b; b.build(force=False)"
for r in 1 2 3; do
  step d20 120 python bench.py --steps 20 --warmup 5 --no-eval >> $O/d20.jsonl
  step g10 120 python bench.py --steps 20 --warmup 5 --no-eval --graph-group 10 >> $O/g10.jsonl
  step g20 120 python bench.py --steps 20 --warmup 5 --no-eval --graph-group 20 >> $O/g20.jsonl
  step d200 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/d200.jsonl
done
python3 -c "
import json, statistics as st
for f in ('d20','g10','g20','d200'):
    recs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    ms = [r['ms_per_step'] for r in recs]; ev = [r.get('gpu_event_ms_per_step') for r in recs]
    print(f, 'host', ms, 'median', st.median(ms), 'events', ev)"
