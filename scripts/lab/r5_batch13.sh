#!/bin/bash
# round 5, GPU batch 13: the headline step as two 4-model pipelines on two streams of one graph
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b13
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
step probe1 180 python scripts/lab/two_stream_probe.py > $O/probe1.jsonl
cat $O/probe1.jsonl
step probe2 180 python scripts/lab/two_stream_probe.py > $O/probe2.jsonl
cat $O/probe2.jsonl
(cd /tmp && step prof 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 $R/scripts/lab/two_stream_probe.py > $O/prof.log 2>&1) || exit 1
ls $O/prof
