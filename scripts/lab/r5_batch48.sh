#!/bin/bash
# round 5, GPU batch 48: top-k GPU tests after the GEMM-decode split refactor; smoke
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b48
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
step tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "topk" > $O/tests.log 2>&1
tail -1 $O/tests.log
step smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
