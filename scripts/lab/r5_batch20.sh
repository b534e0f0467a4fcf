#!/bin/bash
# round 5, GPU batch 20: the driver's 20 / 5 command with 5-step (default), 10-step and 20-step graphs,
# six interleaved runs each (batch 6 hinted at 10-step graphs being ~1 % faster)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b20
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
step tests 300 python -u -m pytest tests/test_bench_gpu.py -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
for r in 1 2 3 4 5 6; do
  step g5 120 python bench.py --steps 20 --warmup 5 --no-eval >> $O/g5.jsonl
  step g10 120 python bench.py --steps 20 --warmup 5 --no-eval --graph-group 10 >> $O/g10.jsonl
  step g20 120 python bench.py --steps 20 --warmup 5 --no-eval --graph-group 20 >> $O/g20.jsonl
done
python3 -c "
import json, statistics as st
for f in ('g5','g10','g20'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    ms = [r['ms_per_step'] for r in rs]; ev = [r['gpu_event_ms_per_step'] for r in rs]
    print(f, ms, 'median', st.median(ms), 'events median', st.median(ev))"
