#!/bin/bash
# round 5, GPU batch 4: candidate top-k after the first optimisation pass (A/B vs dense + profile),
# pipelined BK32 A/B on the headline step, GEMM phase stamps (raw ticks)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b4
mkdir -p $O/phases
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[batch] $name: $*" >&2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "[batch] $name rc=$rc" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[batch] stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
step build 600 python -c "from sparse_coding__amd.ops import build as b; b.build(force=False)"
step test 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py -q -k "topk or sae_epilogues or fused_step_matches" --timeout 120 --timeout-method thread > $O/test.log 2>&1
tail -4 $O/test.log
for r in 1 2; do
  for v in dense cand; do
    SC_TOPK_SELECT=$v step topk_$v 200 python scripts/bench_configs.py topk --steps 80 --warmup 16 >> $O/topk_$v.jsonl
  done
done
python3 -c "
import json
for v in ('dense','cand'):
    print(v, [json.loads(l)['ms_per_step'] for l in open('$O/topk_'+v+'.jsonl') if l.startswith('{')])"
(cd /tmp && SC_TOPK_SELECT=cand step prof_topk 300 rocprofv3 --kernel-trace --stats -d $O/prof_topk -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py topk --steps 40 --warmup 8 > $O/prof_topk.log 2>&1)
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r5b4/prof_topk/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(f"{r['Name'][:100]:100s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us")
PY
for r in 1 2 3 4; do
  step base 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/base.jsonl
  SC_GEMM_CFG="0:29,6:29,7:29" step p32all 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/p32all.jsonl
  SC_GEMM_CFG="7:29" step p32dc 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/p32dc.jsonl
  SC_GEMM_CFG="0:29,6:29" step p32enc 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/p32enc.jsonl
done
python3 -c "
import json, statistics as st
for f in ('base','p32all','p32dc','p32enc'):
    ms = [json.loads(l)['ms_per_step'] for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, ms, 'median', st.median(ms))"
step phases 120 scripts/lab/gemm_phases_128 $O/phases > $O/phases.jsonl
python3 scripts/lab/phase_budget.py $O/phases > $O/phase_budget.txt; cat $O/phase_budget.txt
