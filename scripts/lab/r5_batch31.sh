#!/bin/bash
# round 5, GPU batch 31: kernel budgets of config 4 with the large-k GEMM decode (SC_TOPK_GEMM_K=96)
# and without (0)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b31
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
for gk in 96 0; do
  (cd /tmp && SC_TOPK_GEMM_K=$gk step prof$gk 300 rocprofv3 --kernel-trace --stats -d $O/prof$gk -o run --output-format csv -- python3 $R/scripts/bench_configs.py topk --steps 96 --warmup 16 > $O/prof$gk.log 2>&1) || exit 1
  python3 scripts/lab/step_budget.py $O/prof$gk 800 > $O/step_budget_tk$gk.txt 2>&1
  cat $O/step_budget_tk$gk.txt
done
