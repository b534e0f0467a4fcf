#!/bin/bash
# Iteration loop on the GPU box: build, kernel tests, kernel timings, bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m sparse_coding__amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/ -m gpu -x -q > gpurun_out/gputests.log 2>&1; rc=$?
tail -15 gpurun_out/gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kernel_bench.py ${KB_ARGS} > gpurun_out/kbench.jsonl 2> gpurun_out/kbench.err || { tail -20 gpurun_out/kbench.err; exit 1; }
cat gpurun_out/kbench.jsonl
timeout -k 10 300 python bench.py --steps 100 --warmup 10 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
