#!/bin/bash
# round 5, GPU batch 9: per-kernel step budgets of the current tree (headline + config-4 top-k, rocprofv3
# kernel trace), GEMM configuration A/B for the top-k weight gradient / scores and the masked ensemble
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b9
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
(cd /tmp && step prof_head 300 rocprofv3 --kernel-trace --stats -d $O/prof_head -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --no-eval > $O/prof_head.log 2>&1) || exit 1
python3 scripts/lab/step_budget.py $O/prof_head 1200 > $O/step_budget_head.txt; cat $O/step_budget_head.txt
(cd /tmp && step prof_topk 300 rocprofv3 --kernel-trace --stats -d $O/prof_topk -o run --output-format csv -- python3 $R/scripts/bench_configs.py topk --steps 96 --warmup 16 > $O/prof_topk.log 2>&1) || exit 1
python3 scripts/lab/step_budget.py $O/prof_topk 800 > $O/step_budget_topk.txt; cat $O/step_budget_topk.txt
for r in 1 2; do
  step tk 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/tk.jsonl
  SC_GEMM_CFG="4:25" step tk_wg25 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/tk_wg25.jsonl
  SC_GEMM_CFG="4:13" step tk_wg13 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/tk_wg13.jsonl
  SC_GEMM_CFG="3:29" step tk_sc29 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/tk_sc29.jsonl
  step mk 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/mk.jsonl
  SC_GEMM_CFG="0:25,6:25,7:25" step mk25 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/mk25.jsonl
  SC_GEMM_CFG="0:13,6:13,7:13" step mk13 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/mk13.jsonl
done
python3 -c "
import json, statistics as st
for f in ('tk','tk_wg25','tk_wg13','tk_sc29'):
    ms = [json.loads(l)['ms_per_step'] for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, ms)
for f in ('mk','mk25','mk13'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, [(r['masked_ms_per_step'], r['unmasked_ms_per_step'], r['time_ratio']) for r in rs])"
