#!/bin/bash
# round 5, GPU batch 3: split-tail test, GEMM phase stamps (fixed), split-tail A/B on the headline bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b3
mkdir -p $O/phases
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[batch] $name: $*" >&2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "[batch] $name rc=$rc" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[batch] stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
# the snapshot may be taken mid-edit: rebuild in-tree when the sources are newer than the library
step build 600 python -c "from sparse_coding__amd.ops import build as b; b.build(force=False)"
step test 400 python -u -m pytest tests/test_graphs_gpu.py tests/test_kernels_gpu.py -q -k "split_tail or multi_step or fused_step_tail or topk or sae_epilogues or fused_step_matches" --timeout 120 --timeout-method thread > $O/test.log 2>&1
tail -30 $O/test.log
for r in 1 2; do
  for v in dense cand; do
    SC_TOPK_SELECT=$v step topk_$v 200 python scripts/bench_configs.py topk --steps 80 --warmup 16 >> $O/topk_$v.jsonl
  done
done
cat $O/topk_*.jsonl
(cd /tmp && SC_TOPK_SELECT=cand step prof_topk 300 rocprofv3 --kernel-trace --stats -d $O/prof_topk -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py topk --steps 40 --warmup 8 > $O/prof_topk.log 2>&1)
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r5b3/prof_topk/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{r['Name'][:110]:110s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us {float(r['Percentage']):6.2f}%")
PY
for r in 1 2 3; do
  for v in 0 1; do
    SC_SPLIT_TAIL=$v step ab_$v 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/ab_$v.jsonl
  done
  SC_GEMM_CFG="0:14,7:14" step cfg14 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/cfg14.jsonl
  SC_GEMM_CFG="0:14,6:14,7:14" step cfg14c 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/cfg14c.jsonl
  SC_GEMM_CFG="0:14,7:14" SC_SPLIT_TAIL=1 step cfg14s 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/cfg14s.jsonl
  SC_GEMM_CFG="0:29,6:29,7:29" step cfg29 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/cfg29.jsonl
  SC_GEMM_CFG="0:29,6:29,7:29" SC_SPLIT_TAIL=1 step cfg29s 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/cfg29s.jsonl
done
python3 - <<'PY'
import json
for f in ("cfg14", "cfg14c", "cfg14s", "cfg29", "cfg29s"):
    ms = [json.loads(l)["ms_per_step"] for l in open(f"gpurun_out/r5b3/{f}.jsonl") if l.startswith("{")]
    print(f, ms)
PY
for r in 1 2; do
  for v in 0 1; do
    SC_SPLIT_TAIL=$v step drv_$v 120 python bench.py --steps 20 --warmup 5 --no-eval >> $O/drv_$v.jsonl
  done
done
python3 - <<'PY'
import json
for v in (0, 1):
    for f in ("ab", "drv"):
        ms = [json.loads(l)["ms_per_step"] for l in open(f"gpurun_out/r5b3/{f}_{v}.jsonl") if l.startswith("{")]
        print(f"split={v} {f}: {ms}")
PY
step masked_test 300 python -u -m pytest tests/test_masked_gpu.py -q --timeout 120 --timeout-method thread > $O/masked_test.log 2>&1
tail -3 $O/masked_test.log
for r in 1 2; do
  step masked_base 200 python scripts/bench_configs.py masked --steps 80 --warmup 16 >> $O/masked_base.jsonl
  SC_MASKED_DEC_CFG=5 step masked_lpt5 200 python scripts/bench_configs.py masked --steps 80 --warmup 16 --variant masked >> $O/masked_lpt5.jsonl
done
cat $O/masked_*.jsonl
