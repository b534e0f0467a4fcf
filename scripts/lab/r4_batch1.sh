#!/bin/bash
# Round-4 GPU batch: fused-tail / bf16-gradient A/B + driver command, PMC passes, then the RCCL
# communicator probe (last: it may crash).
set -e
cd "$GRAFT_REPO_ROOT"
bash scripts/lab/tail_ab.sh
bash scripts/gpu.sh pmc > gpurun_out/pmc_step.log 2>&1 || { tail -20 gpurun_out/pmc_step.log; exit 1; }
tail -3 gpurun_out/pmc_step.log
NCCL_DEBUG=WARN timeout -k 10 120 python3 -X faulthandler scripts/lab/rccl_probe.py > gpurun_out/rccl_probe.log 2>&1; echo "probe rc=$?"
tail -30 gpurun_out/rccl_probe.log
