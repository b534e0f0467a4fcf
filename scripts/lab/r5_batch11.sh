#!/bin/bash
# round 5, GPU batch 11: 128x128 BK32 rings for the top-k bf16 GEMMs (scores: layout 3; dense weight
# gradient: layout 0), per-layout SC_GEMM_CFG overrides
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b11
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
step ktest 400 python -u -m pytest tests/test_kernels_gpu.py -q -k "bf16_epilogue_on_bk32 or topk or matmul_layouts" --timeout 120 --timeout-method thread > $O/ktest.log 2>&1
tail -3 $O/ktest.log
for r in 1 2 3; do
  step tk 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/tk.jsonl
  SC_GEMM_CFG="4/3:29" step sc29 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/sc29.jsonl
  SC_GEMM_CFG="4/3:13" step sc13 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/sc13.jsonl
  SC_GEMM_CFG="4/0:25" step wg25 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/wg25.jsonl
  SC_GEMM_CFG="4/0:9" step wg9 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/wg9.jsonl
done
python3 -c "
import json, statistics as st
for f in ('tk','sc29','sc13','wg25','wg9'):
    ms = [json.loads(l)['ms_per_step'] for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, ms, 'median', st.median(ms))"
