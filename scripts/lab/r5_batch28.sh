#!/bin/bash
# round 5, GPU batch 28: workgroup placement of the masked decoder (which tiles share a CU)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b28
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
step phases 120 scripts/lab/gemm_phases_masked $O/phases > $O/phases.jsonl
cat $O/phases.jsonl
for k in dec_masked dec_unmasked2560 dec_128 enc_128_bk32x3; do
  echo "== $k"; python3 scripts/lab/placement.py $O/phases/$k.csv
done > $O/placement.txt 2>&1
cat $O/placement.txt
