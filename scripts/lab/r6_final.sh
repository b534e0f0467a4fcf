# Round 6 final validation on one box: GPU suite, smoke, the driver's bench command, a kernel profile,
# then every config (scripts/lab/r6_configs.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu.sh tests smoke || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/drv.json 2> gpurun_out/drv.err || { tail -20 gpurun_out/drv.err; exit 1; }
head -c 400 gpurun_out/drv.json; echo
bash scripts/gpu.sh prof || exit 1
bash scripts/lab/r6_configs.sh || exit 1
