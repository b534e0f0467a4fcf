#!/bin/bash
# round 5, GPU batch 30: top-k decode + code gradients of the large-k models as dense MFMA GEMMs
# (SC_TOPK_GEMM_K): top-k tests, config-4 A/B over the threshold, kernel budget at the best one
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b30
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
step tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py -x -v --timeout 120 \
  --timeout-method thread -k "topk" > $O/tests.log 2>&1
tail -3 $O/tests.log
for r in 1 2; do
  for gk in 0 96 64 48 32; do
    SC_TOPK_GEMM_K=$gk step tk$gk 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/tk$gk.jsonl
  done
done
python3 -c "
import json
for gk in (0, 96, 64, 48, 32):
    rs = [json.loads(l) for l in open('$O/tk%d.jsonl' % gk) if l.startswith('{')]
    print(gk, [r['ms_per_step'] for r in rs])"
SC_TOPK_GEMM_K=48 step prof 200 rocprofv3 --kernel-trace --stats -d $O/prof -o tk48 -- python3 scripts/bench_configs.py topk --steps 96 --warmup 16 > $O/prof.log 2>&1
python3 scripts/lab/step_budget.py $O/prof 800 > $O/step_budget_tk48.txt 2>&1 || true
cat $O/step_budget_tk48.txt | head -30
