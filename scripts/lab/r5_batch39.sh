#!/bin/bash
# round 5, GPU batch 39: decisive same-box A/B of batch 38's epilogue trims (8 alternating runs at
# 20 / 5, 2 at 200 / 20, 3 masked each)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b39
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
    (cd $R/_abtree && step old 120 python bench.py --steps 20 --warmup 5 --no-eval >> $O/old.jsonl) || exit 1
    step new 120 python bench.py --steps 20 --warmup 5 --no-eval >> $O/new.jsonl
  else
    step new 120 python bench.py --steps 20 --warmup 5 --no-eval >> $O/new.jsonl
    (cd $R/_abtree && step old 120 python bench.py --steps 20 --warmup 5 --no-eval >> $O/old.jsonl) || exit 1
  fi
done
for r in 1 2; do
  step new200 150 python bench.py --steps 200 --warmup 20 --no-eval >> $O/new200.jsonl
  (cd $R/_abtree && step old200 150 python bench.py --steps 200 --warmup 20 --no-eval >> $O/old200.jsonl) || exit 1
done
for r in 1 2 3; do
  step mk_new 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/mk_new.jsonl
  (cd $R/_abtree && step mk_old 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/mk_old.jsonl) || exit 1
done
python3 -c "
import json, statistics as st
for f in ('new','old','new200','old200'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    ms = [r['ms_per_step'] for r in rs]; ev = [r['gpu_event_ms_per_step'] for r in rs]
    print(f, ms, 'median', st.median(ms), 'mean', round(st.mean(ms), 4), 'events median', st.median(ev))
for f in ('mk_new','mk_old'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, [(r['masked_ms_per_step'], r['unmasked_ms_per_step'], r['time_ratio']) for r in rs])"
