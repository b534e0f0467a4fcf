#!/bin/bash
# N>1 rehearsal of bench.py on the one-GPU box: 2 and 4 gloo ranks sharing cuda:0 (ES headline + DP alt)
set -e
mkdir -p gpurun_out/reh
export HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29611 \
    bench.py --gpus $n --steps 10 --warmup 3 --no-eval --dist-backend gloo --shared-gpu > gpurun_out/reh/n$n.json 2> gpurun_out/reh/n$n.err || { tail -30 gpurun_out/reh/n$n.err; exit 1; }
  cat gpurun_out/reh/n$n.json
done
