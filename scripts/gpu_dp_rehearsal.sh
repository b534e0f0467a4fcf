#!/bin/bash
# Rehearse the multi-rank bench path on a 1-GPU box: 2 ranks share cuda:0 over gloo.
# (The real N>1 runs use RCCL on an 8-GPU node; this checks the control flow + JSON.)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --dist-backend gloo --shared-gpu --ring-rows 262144 \
  > gpurun_out/bench_dp2_rehearsal.json 2> gpurun_out/bench_dp2_rehearsal.err || { tail -30 gpurun_out/bench_dp2_rehearsal.err; exit 1; }
cat gpurun_out/bench_dp2_rehearsal.json
