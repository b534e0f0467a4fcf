#!/bin/bash
# round 5, GPU batch 2: step kernel budget (rocprofv3), per-workgroup GEMM phase stamps at the
# production configs, bf16-vs-fp32 quality pin (3000 steps each), quality + kernel tests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b2
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
step phases 120 scripts/lab/gemm_phases_128 $O/phases > $O/phases.jsonl
cat $O/phases.jsonl
(cd /tmp && step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 --no-eval > $O/prof.log 2>&1)
python3 scripts/lab/step_budget.py $O/prof 1200 > $O/step_budget.txt; cat $O/step_budget.txt
step q_fused 240 python bench.py --steps 20 --warmup 5 --quality-steps 3000 > $O/q_fused.json
step q_eager 400 python bench.py --engine eager --steps 20 --warmup 5 --quality-steps 3000 > $O/q_eager.json
step tests 400 python -u -m pytest tests/test_quality_gpu.py tests/test_kernels_gpu.py -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
tail -5 $O/tests.log
