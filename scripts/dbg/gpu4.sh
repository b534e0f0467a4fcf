cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
SC_GEMM_DBG=0 timeout -k 10 200 python -u scripts/dbg/store_lab.py > gpurun_out/store0.log 2>&1 || exit 1
SC_GEMM_DBG=1 timeout -k 10 200 python -u scripts/dbg/store_lab.py > gpurun_out/store1.log 2>&1 || exit 1
grep case gpurun_out/store0.log gpurun_out/store1.log
