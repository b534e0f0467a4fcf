#!/bin/bash
# Full GPU suite + smoke on the current tree.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4suite"; mkdir -p "$O"
bash scripts/gpu.sh tests smoke > "$O/suite.log" 2>&1 || { tail -40 "$O/suite.log"; exit 1; }
grep -E "passed|failed|smoke ok" "$O/suite.log" | tail -3
