#!/bin/bash
# round 5, GPU batch 47: decoder on the pipelined BK32 rings without the early x-tile prefetch (its 32
# registers made the pipelined decoder spill): tests, isolated, step and masked A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b47
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
tail -1 $O/tests.log
step lab 300 python scripts/gemm_lab.py --rounds 5 --which step_dec --cfgs 1,29,25 --out $O/lab.jsonl > $O/lab.log 2>&1
cat $O/lab.jsonl
for r in 1 2 3; do
  step base 120 env SC_GEMM_CFG= python bench.py --steps 20 --warmup 5 --no-eval >> $O/base.jsonl
  step d29 120 env SC_GEMM_CFG=1:29 python bench.py --steps 20 --warmup 5 --no-eval >> $O/d29.jsonl
  step d25 120 env SC_GEMM_CFG=1:25 python bench.py --steps 20 --warmup 5 --no-eval >> $O/d25.jsonl
done
for r in 1 2; do
  step mk_base 200 env SC_GEMM_CFG= python scripts/bench_configs.py masked --steps 200 --warmup 16 --variant masked >> $O/mk_base.jsonl
  step mk_d29 200 env SC_GEMM_CFG=1:29 python scripts/bench_configs.py masked --steps 200 --warmup 16 --variant masked >> $O/mk_d29.jsonl
done
python3 -c "
import json, statistics as st
for f in ('base','d29','d25'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    ms = [r['ms_per_step'] for r in rs]
    print(f, ms, 'median', st.median(ms))
for f in ('mk_base','mk_d29'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, [r['masked_ms_per_step'] for r in rs])"
