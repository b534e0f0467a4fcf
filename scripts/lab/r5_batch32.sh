#!/bin/bash
# round 5, GPU batch 32: which hipBLASLt kernels torch.matmul picks at the step's GEMM shapes (kernel
# names carry the macro tile / MFMA / depth), timed beside ours
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b32
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
step lab 300 python scripts/gemm_lab.py --rounds 5 --which step_torch,step_enc,step_dec,step_dc,step_wgrad --cfgs 1,29 --out $O/lab.jsonl > $O/lab.log 2>&1
cat $O/lab.jsonl
(cd /tmp && step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/scripts/gemm_lab.py --rounds 1 --which step_torch --out $O/lab_prof.jsonl > $O/prof.log 2>&1) || exit 1
python3 - <<PY
import csv, glob, collections
f = glob.glob("$O/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r.get("Name", "")[:300], r.get("Calls"), r.get("AverageNs"))
PY
