set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6_fista
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fista" > gpurun_out/r6_fista/test.log 2>&1 || { tail -40 gpurun_out/r6_fista/test.log; exit 1; }
tail -3 gpurun_out/r6_fista/test.log
timeout -k 10 400 python -u scripts/fista_step_ab.py --rounds 3 --steps 15 > gpurun_out/r6_fista/ab.json 2> gpurun_out/r6_fista/ab.err || { tail -30 gpurun_out/r6_fista/ab.err; exit 1; }
cat gpurun_out/r6_fista/ab.json
