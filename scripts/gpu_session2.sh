#!/bin/bash
# Ensemble-sharding validation: GPU tests, N=1 bench, RCCL single-rank rehearsal of the
# sharded path, 2-rank gloo shared-GPU rehearsal, per-N projection.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?
tail -8 gpurun_out/gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --force-dist --steps 100 --warmup 10 > gpurun_out/bench_es1_rccl.json 2> gpurun_out/bench_es1_rccl.err || { tail -30 gpurun_out/bench_es1_rccl.err; exit 1; }
cat gpurun_out/bench_es1_rccl.json
timeout -k 10 300 python scripts/es_projection.py > gpurun_out/es_projection.jsonl 2> gpurun_out/es_projection.err || { tail -20 gpurun_out/es_projection.err; exit 1; }
cat gpurun_out/es_projection.jsonl
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 2 --steps 20 --warmup 3 --dist-backend gloo --shared-gpu --ring-rows 262144 > gpurun_out/bench_es2_gloo.json 2> gpurun_out/bench_es2_gloo.err || { tail -30 gpurun_out/bench_es2_gloo.err; exit 1; }
cat gpurun_out/bench_es2_gloo.json
