cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
for D in 0 1; do
  rm -rf gpurun_out/tr$D
  (cd /tmp && SC_GEMM_DBG=$D timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/tr$D -o run --output-format csv -- python3 $R/scripts/dbg/trace_lab.py > $R/gpurun_out/tr$D.log 2>&1) || { tail -5 gpurun_out/tr$D.log; exit 1; }
  python3 scripts/dbg/trace_split.py gpurun_out/tr$D.log gpurun_out/tr$D $D
done
timeout -k 10 120 python -u scripts/dbg/ramp2.py > gpurun_out/ramp2.log 2>&1; echo "ramp2 rc=$?"; cat gpurun_out/ramp2.log | grep -v amdgpu.ids
