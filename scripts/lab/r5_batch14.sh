#!/bin/bash
# round 5, GPU batch 14: 256x256 blocks (two full rounds instead of 2.67) with the BK32 rings for the
# encoder / code gradient, in the step
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b14
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
for r in 1 2 3; do
  step base 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/base.jsonl
  SC_GEMM_CFG="0:7,6:7,7:7" step s256x4 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/s256x4.jsonl
  SC_GEMM_CFG="0:15,6:15,7:15" step s256x3 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/s256x3.jsonl
  SC_GEMM_CFG="0:3,6:3,7:3" step s256 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/s256.jsonl
done
python3 -c "
import json, statistics as st
for f in ('base','s256x4','s256x3','s256'):
    ms = [json.loads(l)['ms_per_step'] for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, ms, 'median', st.median(ms))"
