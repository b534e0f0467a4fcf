#!/bin/bash
# round 5, GPU batch 34: 256x128 blocks (four 128x64 waves, hipBLASLt's macro tile for these shapes)
# with the software-pipelined BK64 K loop, VGPR-form accumulators: tests, isolated GEMMs, step A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b34
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
step tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_headline_grad_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "matmul_layouts or sae_epilogues or headline or weight_grads or code_grad or decode" > $O/tests.log 2>&1
tail -2 $O/tests.log
step lab 300 python scripts/gemm_lab.py --rounds 5 --which step_torch,step_enc,step_dec,step_dc --cfgs 1,29,2 --out $O/lab.jsonl > $O/lab.log 2>&1
cat $O/lab.jsonl
run() {  # name cfg
  local name=$1; shift
  step $name 120 env SC_GEMM_CFG="$1" python bench.py --steps 20 --warmup 5 --no-eval >> $O/$name.jsonl
}
for r in 1 2 3; do
  run base ""
  run enc2 "0:2,6:2,7:2"
  run dec2 "1:2"
  run all2 "0:2,6:2,7:2,1:2"
done
python3 -c "
import json, statistics as st
for f in ('base','enc2','dec2','all2'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    ms = [r['ms_per_step'] for r in rs]
    print(f, ms, 'median', st.median(ms))"
