#!/bin/bash
# round 5, GPU batch 26: fused encoder + decoder launch (SC_FUSED_ENCDEC=1): bit-equality against the
# two launches, then step A/B at the driver's 20 / 5 (decoder BK64 x 2 and BK32 x 3, 4 runs each,
# order rotated per round)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b26
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
step test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k fused_encdec > $O/tests.log 2>&1
run() {  # name env...
  local name=$1; shift
  step $name 120 env "$@" python bench.py --steps 20 --warmup 5 --no-eval >> $O/$name.jsonl
}
for r in 1 2 3 4; do
  if [ $((r % 2)) -eq 0 ]; then
    run fused SC_FUSED_ENCDEC=1; run base SC_FUSED_ENCDEC=0
    run fused13 SC_FUSED_ENCDEC=1 SC_GEMM_CFG=1:13; run base13 SC_FUSED_ENCDEC=0 SC_GEMM_CFG=1:13
  else
    run base SC_FUSED_ENCDEC=0; run fused SC_FUSED_ENCDEC=1
    run base13 SC_FUSED_ENCDEC=0 SC_GEMM_CFG=1:13; run fused13 SC_FUSED_ENCDEC=1 SC_GEMM_CFG=1:13
  fi
done
python3 -c "
import json, statistics as st
for f in ('base','fused','base13','fused13'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    ms = [r['ms_per_step'] for r in rs]; ev = [r['gpu_event_ms_per_step'] for r in rs]
    print(f, ms, 'median', st.median(ms), 'events median', st.median(ev))"
