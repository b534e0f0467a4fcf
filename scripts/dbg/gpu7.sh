cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
export SC_GEMM_DBG=1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1)); rm -rf gpurun_out/pm$i
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $P -d $R/gpurun_out/pm$i -o run --output-format csv -- python3 $R/scripts/dbg/trace_lab.py > $R/gpurun_out/pm$i.log 2>&1) || { tail -5 gpurun_out/pm$i.log; echo "pass $i failed"; continue; }
  python3 scripts/dbg/pmc_split.py gpurun_out/pm$i.log gpurun_out/pm$i
done
unset SC_GEMM_DBG
timeout -k 10 300 python -u -m pytest tests/test_gemm_persistent_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pers.log 2>&1; echo "pers rc=$?"; tail -3 gpurun_out/pers.log
