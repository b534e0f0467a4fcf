#!/bin/bash
# round 5, GPU batch 22: decisive A/B of the graph group at the driver's 20 / 5 (8 runs each, order
# alternating per round)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b22
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
for r in 1 2 3 4 5 6 7 8; do
  if [ $((r % 2)) -eq 0 ]; then
    step g10 120 python bench.py --steps 20 --warmup 5 --no-eval --graph-group 10 >> $O/g10.jsonl
    step g5 120 python bench.py --steps 20 --warmup 5 --no-eval --graph-group 5 >> $O/g5.jsonl
  else
    step g5 120 python bench.py --steps 20 --warmup 5 --no-eval --graph-group 5 >> $O/g5.jsonl
    step g10 120 python bench.py --steps 20 --warmup 5 --no-eval --graph-group 10 >> $O/g10.jsonl
  fi
done
python3 -c "
import json, statistics as st
for f in ('g5','g10'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    ms = [r['ms_per_step'] for r in rs]; ev = [r['gpu_event_ms_per_step'] for r in rs]
    print(f, ms, 'median', st.median(ms), 'mean', round(st.mean(ms), 4), 'events median', st.median(ev))"
