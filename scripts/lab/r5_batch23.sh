#!/bin/bash
# round 5, GPU batch 23: wave-per-row bf16 top-k select (tests + config-4 A/B against the block select)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b23
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
step ktest 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py -q -k "topk" --timeout 120 --timeout-method thread > $O/ktest.log 2>&1
tail -3 $O/ktest.log
for r in 1 2 3; do
  step wave 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/wave.jsonl
  SC_TOPK_SELECT=block step block 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/block.jsonl
done
(cd /tmp && step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/scripts/bench_configs.py topk --steps 96 --warmup 16 > $O/prof.log 2>&1) || exit 1
python3 scripts/lab/step_budget.py $O/prof 800 > $O/step_budget_topk.txt; cat $O/step_budget_topk.txt
python3 -c "
import json, statistics as st
for f in ('wave','block'):
    ms = [json.loads(l)['ms_per_step'] for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, ms, 'median', st.median(ms))"
