#!/bin/bash
# round 5, GPU batch 35: plain bf16 NT GEMM at the encoder shape, 128x128 vs 256x128 vs hipBLASLt, and
# phase stamps of the 256x128 blocks (main loop vs epilogue)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b35
mkdir -p $O/phases
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
step lab 300 python scripts/gemm_lab.py --rounds 5 --which step_torch_enc,step_ntbf16,step_enc --cfgs 1,29,2 --out $O/lab.jsonl > $O/lab.log 2>&1
cat $O/lab.jsonl
step phases 120 scripts/lab/gemm_phases_256x128 $O/phases > $O/phases.jsonl
python3 scripts/lab/phase_budget.py $O/phases 1 > $O/phase_budget.txt 2>&1
cat $O/phase_budget.txt
