set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_persistent_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pers.log 2>&1; echo "pers rc=$?"; grep -E "passed|failed|FAIL" gpurun_out/pers.log | tail -8
timeout -k 10 400 python -u scripts/gemm_lab.py --which step_ --cfgs 1,5,3 --out gpurun_out/gemm_lab.jsonl > gpurun_out/gemm_lab.log 2>&1; echo "lab rc=$?"; cat gpurun_out/gemm_lab.log
