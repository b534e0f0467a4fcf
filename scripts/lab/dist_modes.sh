# One-rank RCCL rehearsal of bench.py's distributed modes (the driver runs N = 1..8 itself).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for mode in dp zero1 es; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --force-dist --parallelism $mode --steps 50 --warmup 10 --no-eval \
    > gpurun_out/dist_$mode.json 2> gpurun_out/dist_$mode.err || { tail -20 gpurun_out/dist_$mode.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/dist_$mode.json').read().strip().splitlines()[-1]); print('$mode', d['ms_per_step'], d['config']['parallelism'], d.get('comm_bytes_per_gpu_per_step'))"
done
