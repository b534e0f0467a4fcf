# Round 6 end: every BASELINE config / engine on the final tree, one box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_configs; rm -rf $O; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "[cfg] $name" >&2; timeout -k 10 "$t" "$@" > $O/$name.json 2>> $O/err.log || { echo "[cfg] $name failed"; tail -20 $O/err.log; exit 1; }; cat $O/$name.json; }
step drv 200 python bench.py --steps 20 --warmup 5
step b200 200 python bench.py --steps 200 --warmup 20 --no-eval
step topk 200 python scripts/bench_configs.py topk --steps 200 --warmup 16
step masked 200 python scripts/bench_configs.py masked --steps 200 --warmup 16
step fistaloss 300 python scripts/bench_configs.py fistaloss --steps 10 --warmup 2
step fista 300 python scripts/bench_configs.py fista --steps 10 --warmup 2
step mlpout 300 python scripts/bench_configs.py mlpout --steps 50 --warmup 10
step lista 200 python scripts/unrolled_bench.py
step residual 200 python scripts/unrolled_bench.py --residual
step eager 300 python bench.py --engine eager --steps 20 --warmup 5 --no-eval
