#!/bin/bash
# round 5, GPU batch 10: top-k on bf16 scores (select with exact tie resolution): tests, A/B against the
# fp32 score matrix, kernel budget; masked-ensemble GEMM configurations
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b10
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
  step tk_bf 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/tk_bf.jsonl
  SC_TOPK_SCORES=fp32 step tk_f32 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/tk_f32.jsonl
done
(cd /tmp && step prof_topk 300 rocprofv3 --kernel-trace --stats -d $O/prof_topk -o run --output-format csv -- python3 $R/scripts/bench_configs.py topk --steps 96 --warmup 16 > $O/prof_topk.log 2>&1) || exit 1
python3 scripts/lab/step_budget.py $O/prof_topk 800 > $O/step_budget_topk.txt; cat $O/step_budget_topk.txt
for r in 1 2; do
  step mk 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/mk.jsonl
  SC_GEMM_CFG="0:25,6:25,7:25" step mk25 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/mk25.jsonl
  SC_GEMM_CFG="0:13,6:13,7:13" step mk13 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/mk13.jsonl
done
python3 -c "
import json
for f in ('tk_bf','tk_f32'):
    print(f, [json.loads(l)['ms_per_step'] for l in open('$O/'+f+'.jsonl') if l.startswith('{')])
for f in ('mk','mk25','mk13'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, [(r['masked_ms_per_step'], r['unmasked_ms_per_step'], r['time_ratio']) for r in rs])"
