#!/bin/bash
# round 5, GPU batch 5: 128x256 blocks for the K = 512 step GEMMs (A/B vs the pipelined 128x128
# default), then the whole GPU suite, the driver's bench command and smoke on the resulting tree
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b5
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[batch] $name: $*" >&2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "[batch] $name rc=$rc" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[batch] stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
step build 600 python -c "from sparse_coding__amd.ops import build as b; b.build(force=False)"
step ktest 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "sae_epilogues or fused_step_matches" --timeout 120 --timeout-method thread > $O/ktest.log 2>&1
tail -3 $O/ktest.log
for r in 1 2 3 4; do
  step base 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/base.jsonl
  SC_GEMM_CFG="0:45,7:45" step wide 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/wide.jsonl
  SC_GEMM_CFG="0:45" step wide_enc 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/wide_enc.jsonl
  SC_GEMM_CFG="7:45" step wide_dc 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/wide_dc.jsonl
done
python3 -c "
import json, statistics as st
for f in ('base','wide','wide_enc','wide_dc'):
    ms = [json.loads(l)['ms_per_step'] for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, ms, 'median', st.median(ms))"
step suite 500 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/suite.log 2>&1
tail -5 $O/suite.log
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step drv 150 python bench.py --steps 20 --warmup 5 > $O/drv.json
cat $O/drv.json | head -c 400; echo
