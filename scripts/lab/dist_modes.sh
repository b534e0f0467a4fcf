# One-rank RCCL rehearsal of bench.py's distributed modes (the driver runs N = 1..8 itself).
# DIST_MODES: "mode:chunks ..." (default: dp:2 zero1:2 es:1)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for mc in ${DIST_MODES:-dp:2 zero1:2 es:1}; do
  mode=${mc%%:*}; ch=${mc##*:}
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --force-dist --parallelism $mode --dp-chunks $ch --steps 50 --warmup 10 \
    --no-eval > gpurun_out/dist_${mode}_$ch.json 2> gpurun_out/dist_${mode}_$ch.err || { tail -20 gpurun_out/dist_${mode}_$ch.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/dist_${mode}_$ch.json').read().strip().splitlines()[-1]); print('$mode chunks=$ch', d['ms_per_step'], d['config']['parallelism'])"
done
