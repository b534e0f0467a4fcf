#!/bin/bash
# round 5, GPU batch 8: the software-pipelined BK32 K loop (cfg bit 4) on the decoder and the weight
# gradient (128x128 blocks), in the step; bf16 weight-gradient storage (repeats + 3000-step quality run)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b8
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
  SC_GEMM_CFG="1:25" step dec25 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/dec25.jsonl
  SC_GEMM_CFG="1:29" step dec29 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/dec29.jsonl
  SC_GEMM_CFG="3:25" step wg25 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/wg25.jsonl
  SC_GEMM_CFG="3:9" step wg9 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/wg9.jsonl
  step gbf 120 python bench.py --steps 200 --warmup 20 --no-eval --wgrad-dtype bf16 >> $O/gbf.jsonl
done
step q_gbf 300 python bench.py --steps 20 --warmup 5 --quality-steps 3000 --wgrad-dtype bf16 > $O/q_fused_gbf.json
python3 -c "
import json, statistics as st
for f in ('base','dec25','dec29','wg25','wg9','gbf'):
    ms = [json.loads(l)['ms_per_step'] for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, ms, 'median', st.median(ms))"
