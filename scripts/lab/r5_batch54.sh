#!/bin/bash
# round 5, GPU batch 54: decisive same-box A/B of the restructured row Adam (one row per wave, 71 VGPRs,
# 7 waves / SIMD) against the previous commit's tree (_abtree): 8 alternating 20 / 5 runs, 2 x 200 / 20
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b54
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
step tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py tests/test_masked_gpu.py tests/test_headline_grad_gpu.py -x -q \
  --timeout 120 --timeout-method thread -k "adam or tail or masked or fused_step or headline" > $O/tests.log 2>&1
grep -E "passed|failed" $O/tests.log | tail -1
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
python3 -c "
import json, statistics as st
for f in ('new','old','new200','old200'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    ms = [r['ms_per_step'] for r in rs]; ev = [r['gpu_event_ms_per_step'] for r in rs]
    print(f, ms, 'median', st.median(ms), 'mean', round(st.mean(ms), 4), 'events median', st.median(ev))"
