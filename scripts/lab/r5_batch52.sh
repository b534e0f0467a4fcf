#!/bin/bash
# round 5, GPU batch 52: the masked config's step tail split into its separate kernels (SC_FUSED_TAIL=0)
# to see what the row Adam alone costs masked vs unmasked
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b52
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
for v in masked unmasked; do
  (cd /tmp && SC_FUSED_TAIL=0 step prof_$v 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $R/scripts/bench_configs.py masked --variant $v --steps 96 --warmup 16 > $O/prof_$v.log 2>&1) || exit 1
  python3 scripts/lab/step_budget.py $O/prof_$v 800 > $O/step_budget_$v.txt 2>&1
  head -14 $O/step_budget_$v.txt
done
