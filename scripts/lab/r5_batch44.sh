#!/bin/bash
# round 5, GPU batch 44: same-box A/B of the top-k scores GEMM: ours vs hipBLASLt ([B, G, n]) with the
# select in memory order (SC_TOPK_BGN_ORDER=1) or model-rotated (2); 4 alternating runs each
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b44
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
  -k "topk_select_bf16 or library_scores" > $O/tests.log 2>&1
tail -1 $O/tests.log
for r in 1 2 3 4; do
  SC_TOPK_SCORES_GEMM=sc step sc 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/sc.jsonl
  SC_TOPK_SCORES_GEMM=blas SC_TOPK_BGN_ORDER=1 step blas1 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/blas1.jsonl
  SC_TOPK_SCORES_GEMM=blas SC_TOPK_BGN_ORDER=2 step blas2 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/blas2.jsonl
done
python3 -c "
import json, statistics as st
for f in ('sc', 'blas1', 'blas2'):
    rs = [json.loads(l) for l in open('$O/%s.jsonl' % f) if l.startswith('{')]
    ms = [r['ms_per_step'] for r in rs]
    print(f, ms, 'median', st.median(ms))"
