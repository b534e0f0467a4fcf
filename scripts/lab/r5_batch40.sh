#!/bin/bash
# round 5, GPU batch 40: the other BASELINE configs on the final round-5 tree: config 5 FISTA (small
# ring), FISTA in the loss, Pythia-70m MLP configs, the eager bar
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b40
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
step fista 400 python scripts/bench_configs.py fista --steps 6 --warmup 2 --ratio 1.0 > $O/fista.json
cat $O/fista.json
step fistaloss 300 python scripts/bench_configs.py fistaloss --steps 20 --warmup 5 > $O/fistaloss.json
cat $O/fistaloss.json
step mlp 300 python scripts/bench_configs.py mlp --steps 50 --warmup 10 > $O/mlp.json
cat $O/mlp.json
step mlpout 300 python scripts/bench_configs.py mlpout --steps 50 --warmup 10 > $O/mlpout.json
cat $O/mlpout.json
step eager 300 python bench.py --engine eager --steps 10 --warmup 3 --no-eval > $O/eager.json
head -c 400 $O/eager.json; echo
