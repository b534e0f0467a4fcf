#!/bin/bash
# round 5, GPU batch 7: the fused top-k tail (tests + config-4 A/B) and bf16 weight-gradient storage on
# the headline step
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b7
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
step ktest 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py -q -k "topk" --timeout 120 --timeout-method thread > $O/ktest.log 2>&1
tail -3 $O/ktest.log
for r in 1 2 3; do
  step tk_tail 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/tk_tail.jsonl
  SC_TOPK_TAIL=0 step tk_split 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/tk_split.jsonl
  step base 120 python bench.py --steps 200 --warmup 20 --no-eval >> $O/base.jsonl
  step gbf 120 python bench.py --steps 200 --warmup 20 --no-eval --wgrad-dtype bf16 >> $O/gbf.jsonl
done
python3 -c "
import json, statistics as st
for f in ('tk_tail','tk_split','base','gbf'):
    ms = [json.loads(l)['ms_per_step'] for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, ms, 'median', st.median(ms))"
