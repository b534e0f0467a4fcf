#!/bin/bash
# round 5, GPU batch 55: end to end on the final tree (harvest -> HBM ring -> fused 8-model sweep ->
# FVU / L0 -> reference-layout checkpoint round trip), 20k steps as in round 4
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b55
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
step e2e 600 python -u scripts/e2e_pythia70m.py --rows 2000000 --steps 20000 --out $O > $O/e2e.log 2>&1
tail -5 $O/e2e.log
