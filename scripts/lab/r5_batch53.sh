#!/bin/bash
# round 5, GPU batch 53: row Adam restructured (all rows' loads first; 1 or 2 rows per wave,
# SC_ADAM_RPW): tests, then same-box A/B against the previous commit's tree (_abtree) -- headline
# and masked
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b53
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
step tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py tests/test_masked_gpu.py -x -q \
  --timeout 120 --timeout-method thread -k "adam or tail or masked or fused_step" > $O/tests.log 2>&1
grep -E "passed|failed" $O/tests.log | tail -1
step tests2 400 env SC_ADAM_RPW=2 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py tests/test_masked_gpu.py -x -q \
  --timeout 120 --timeout-method thread -k "adam or tail or masked or fused_step" > $O/tests2.log 2>&1
grep -E "passed|failed" $O/tests2.log | tail -1
for r in 1 2 3 4; do
  step r1 120 env SC_ADAM_RPW=1 python bench.py --steps 20 --warmup 5 --no-eval >> $O/r1.jsonl
  step r2 120 env SC_ADAM_RPW=2 python bench.py --steps 20 --warmup 5 --no-eval >> $O/r2.jsonl
  (cd $R/_abtree && step old 120 python bench.py --steps 20 --warmup 5 --no-eval >> $O/old.jsonl) || exit 1
done
for r in 1 2; do
  step mk_r1 200 env SC_ADAM_RPW=1 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/mk_r1.jsonl
  step mk_r2 200 env SC_ADAM_RPW=2 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/mk_r2.jsonl
  (cd $R/_abtree && step mk_old 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/mk_old.jsonl) || exit 1
done
python3 -c "
import json, statistics as st
for f in ('r1','r2','old'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    ms = [r['ms_per_step'] for r in rs]
    print(f, ms, 'median', st.median(ms), 'mean', round(st.mean(ms), 4))
for f in ('mk_r1','mk_r2','mk_old'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, [(r['masked_ms_per_step'], r['unmasked_ms_per_step'], r['time_ratio']) for r in rs])"
