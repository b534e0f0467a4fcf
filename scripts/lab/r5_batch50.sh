#!/bin/bash
# round 5, GPU batch 50: whole GPU suite, smoke, the driver's bench command and 200/20, on the current tree
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b50
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
step suite 700 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/suite.log 2>&1
tail -5 $O/suite.log
step smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
step drv 150 python bench.py --steps 20 --warmup 5 > $O/drv.json
head -c 600 $O/drv.json; echo
step b200 150 python bench.py --steps 200 --warmup 20 > $O/b200.json
head -c 300 $O/b200.json; echo
step topk 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 > $O/topk.json
cat $O/topk.json
step masked 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 > $O/masked.json
cat $O/masked.json
