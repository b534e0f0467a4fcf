set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/dbg/ramp.py > gpurun_out/ramp.log 2>&1; echo "ramp rc=$?"; cat gpurun_out/ramp.log | tail -20
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/kernels.log 2>&1; rc=$?; tail -15 gpurun_out/kernels.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u scripts/gemm_lab.py --which step_ --cfgs 1,5,3 --out gpurun_out/gemm_lab.jsonl > gpurun_out/gemm_lab.log 2>&1; echo "lab rc=$?"; cat gpurun_out/gemm_lab.log
