#!/bin/bash
# end-to-end pipeline run (harvest -> ring -> fused sweep -> FVU/L0 -> checkpoint round trip)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/e2e
timeout -k 10 600 python -u scripts/e2e_pythia70m.py --rows 4000000 --steps 20000 --out gpurun_out/e2e > gpurun_out/e2e/e2e.log 2>&1; rc=$?
tail -c 3000 gpurun_out/e2e/e2e.log
rm -f gpurun_out/e2e/learned_dicts.pt
exit $rc
