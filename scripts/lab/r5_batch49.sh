#!/bin/bash
# round 5, GPU batch 49: 128x128 BK32 x 2 ring (32 KB) held to 128 VGPRs -> FOUR blocks per CU (1024
# slots: the 2048 encoder / code-gradient tiles in two full rounds instead of 2.67 at three per CU)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b49
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
step tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "sae_epilogues or layouts or bk32" > $O/tests.log 2>&1
grep -E "passed|failed" $O/tests.log | tail -1
step lab 300 python scripts/gemm_lab.py --rounds 5 --which step_enc,step_dc --cfgs 29,9 --out $O/lab.jsonl > $O/lab.log 2>&1
cat $O/lab.jsonl
for r in 1 2 3 4; do
  step base 120 env SC_GEMM_CFG= python bench.py --steps 20 --warmup 5 --no-eval >> $O/base.jsonl
  step e9 120 env SC_GEMM_CFG=0:9,7:9 python bench.py --steps 20 --warmup 5 --no-eval >> $O/e9.jsonl
  step enc9 120 env SC_GEMM_CFG=0:9 python bench.py --steps 20 --warmup 5 --no-eval >> $O/enc9.jsonl
done
python3 -c "
import json, statistics as st
for f in ('base','e9','enc9'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    ms = [r['ms_per_step'] for r in rs]
    print(f, ms, 'median', st.median(ms))"
