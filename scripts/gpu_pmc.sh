#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 300 python -m sparse_coding__amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc" -o p1 --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/prof_gemm.py" > "$GRAFT_REPO_ROOT/gpurun_out/pmc1.log" 2>&1 || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/pmc1.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum -d "$GRAFT_REPO_ROOT/gpurun_out/pmc" -o p2 --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/prof_gemm.py" > "$GRAFT_REPO_ROOT/gpurun_out/pmc2.log" 2>&1 || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/pmc2.log"; exit 1; }
ls "$GRAFT_REPO_ROOT/gpurun_out/pmc"
