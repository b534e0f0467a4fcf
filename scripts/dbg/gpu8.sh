cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_pt_gpu.py tests/test_headline_grad_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k8.log 2>&1; rc=$?; tail -4 gpurun_out/k8.log; [ $rc -eq 0 ] || exit 1
for D in 0 1; do
  rm -rf gpurun_out/tr$D
  (cd /tmp && SC_GEMM_DBG=$D timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/tr$D -o run --output-format csv -- python3 $R/scripts/dbg/trace_lab.py > $R/gpurun_out/tr$D.log 2>&1) || { tail -5 gpurun_out/tr$D.log; exit 1; }
  python3 scripts/dbg/trace_split.py gpurun_out/tr$D.log gpurun_out/tr$D $D
done
timeout -k 10 400 python -u scripts/gemm_lab.py --which step_ --cfgs 1,3 --out gpurun_out/gemm_lab.jsonl > gpurun_out/gemm_lab.log 2>&1; echo "lab rc=$?"; grep -v amdgpu gpurun_out/gemm_lab.log
