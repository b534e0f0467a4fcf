#!/bin/bash
# round 5, GPU batch 16: K rotation (cfg bit 6: each tile starts its K walk at (tm + tn) mod nk, so
# blocks sharing an operand panel do not request the same L2 lines in lockstep)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b16
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
step ktest 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_masked_gpu.py -q -k "sae_epilogues or fused_step_matches or compacted" --timeout 120 --timeout-method thread > $O/ktest.log 2>&1
tail -3 $O/ktest.log
for r in 1 2 3; do
  step base 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/base.jsonl
  SC_GEMM_CFG="0:93,6:93,7:93,1:65,3:64" step rot_all 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/rot_all.jsonl
  SC_GEMM_CFG="0:93,6:93,7:93" step rot_encdc 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/rot_encdc.jsonl
  SC_GEMM_CFG="1:65" step rot_dec 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/rot_dec.jsonl
  SC_GEMM_CFG="3:64" step rot_wg 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/rot_wg.jsonl
done
python3 -c "
import json, statistics as st
for f in ('base','rot_all','rot_encdc','rot_dec','rot_wg'):
    ms = [json.loads(l)['ms_per_step'] for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, ms, 'median', st.median(ms))"
