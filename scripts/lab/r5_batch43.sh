#!/bin/bash
# round 5, GPU batch 43: top-k scores as ONE hipBLASLt GEMM over the stacked dictionaries ([B, G, n],
# SC_TOPK_SCORES_GEMM=blas), the select rotating models over XCDs: tests, config-4 A/B, budget
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b43
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
step tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py -x -v --timeout 120 \
  --timeout-method thread -k "topk" > $O/tests.log 2>&1
tail -3 $O/tests.log
for r in 1 2 3; do
  SC_TOPK_SCORES_GEMM=sc step sc 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/sc.jsonl
  SC_TOPK_SCORES_GEMM=blas step blas 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/blas.jsonl
done
python3 -c "
import json
for f in ('sc', 'blas'):
    rs = [json.loads(l) for l in open('$O/%s.jsonl' % f) if l.startswith('{')]
    print(f, [r['ms_per_step'] for r in rs])"
(cd /tmp && SC_TOPK_SCORES_GEMM=blas step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/scripts/bench_configs.py topk --steps 96 --warmup 16 > $O/prof.log 2>&1) || exit 1
python3 scripts/lab/step_budget.py $O/prof 800 > $O/step_budget_blas.txt 2>&1
head -14 $O/step_budget_blas.txt
