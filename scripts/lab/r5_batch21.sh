#!/bin/bash
# round 5, GPU batch 21: the new graph tiling (fewest replays, groups <= 10) -- graph tests, bench tests,
# and the driver's command against the old 5-step tiling
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b21
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
step tests 500 python -u -m pytest tests/test_graphs_gpu.py tests/test_bench_gpu.py tests/test_graphed_multirank_gpu.py tests/test_train_gpu.py -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
for r in 1 2 3 4; do
  step new 120 python bench.py --steps 20 --warmup 5 >> $O/new.jsonl
  step old 120 python bench.py --steps 20 --warmup 5 --graph-group 5 >> $O/old.jsonl
done
step long 150 python bench.py --steps 200 --warmup 20 --no-eval >> $O/long.jsonl
python3 -c "
import json, statistics as st
for f in ('new','old','long'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    ms = [r['ms_per_step'] for r in rs]
    print(f, ms, 'median', st.median(ms))"
