cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_pt_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/pt.log | tail -15
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u scripts/gemm_lab.py --which step_ --cfgs 1,17,21 --out gpurun_out/gemm_lab.jsonl > gpurun_out/gemm_lab.log 2>&1; echo "lab rc=$?"; cat gpurun_out/gemm_lab.log
