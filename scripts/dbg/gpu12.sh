cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py tests/test_gemm_persistent_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k12.log 2>&1; rc=$?; tail -4 gpurun_out/k12.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/bench_configs.py masked --steps 30 --warmup 5 > gpurun_out/masked.json 2> gpurun_out/masked.err; echo "masked rc=$?"; tail -2 gpurun_out/masked.json
timeout -k 10 300 python -u scripts/bench_configs.py mlpout --steps 30 --warmup 5 > gpurun_out/mlpout.json 2> gpurun_out/mlpout.err; echo "mlpout rc=$?"; tail -2 gpurun_out/mlpout.json; tail -3 gpurun_out/mlpout.err
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k fista_dictionary --timeout 120 --timeout-method thread > gpurun_out/fu.log 2>&1; echo "fista-update rc=$?"; tail -3 gpurun_out/fu.log
