set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_dist; mkdir -p $O
echo "=== one-rank RCCL rehearsal (es + alt dp), torchrun"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --force-dist --steps 20 --warmup 5 --no-eval > $O/force_dist.json 2> $O/force_dist.err || { tail -30 $O/force_dist.err; exit 1; }
python3 -c "import json; r=json.loads(open('$O/force_dist.json').read().strip().splitlines()[-1]); print({k: r.get(k) for k in ('ms_per_step','value','predicted_ms_per_step','compute_calibration')}); print(r['collectives']['path'], r['collectives']['fallback'], r.get('alt_parallelism',{}).get('ms_per_step'))"
echo "=== two gloo ranks sharing cuda:0 (launcher path)"
timeout -k 10 400 python bench.py --gpus 2 --shared-gpu --dist-backend gloo --steps 10 --warmup 2 --no-eval --settle-ms 0 > $O/gloo2.json 2> $O/gloo2.err || { tail -30 $O/gloo2.err; exit 1; }
python3 -c "import json; r=json.loads(open('$O/gloo2.json').read().strip().splitlines()[-1]); print({k: r.get(k) for k in ('n_gpus','ms_per_step','compute_calibration')}); print(r['collectives']['path'], r['collectives']['consistency'])"
