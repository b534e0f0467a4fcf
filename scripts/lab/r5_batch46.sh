#!/bin/bash
# round 5, GPU batch 46: weight gradient at 256x128 with the pipelined loop (VGPR form) vs 256x256 / 128x128
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b46
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
step lab 300 python scripts/gemm_lab.py --rounds 5 --which step_wgrad,step_torch_wgrad --cfgs 3,2,1,9 --out $O/lab.jsonl > $O/lab.log 2>&1
cat $O/lab.jsonl
