#!/bin/bash
# round 5, GPU batch 25: PMC of the headline step's kernels inside the bench's own HIP graphs
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b25
mkdir -p $O
python -c "from sparse_coding__amd.ops import build as b; b.build(force=False)" || exit 1
run() {  # name counters...
  local name=$1; shift
  (cd /tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" -d "$O/pmc/$name" -o $name --output-format csv -- python3 $R/bench.py --steps 60 --warmup 20 --no-eval --settle-ms 0 > "$O/$name.log" 2>&1) || { tail -20 "$O/$name.log"; exit 1; }
}
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
ls $O/pmc/p1
run p3 WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
run p4 TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE
python3 scripts/pmc_summary.py $O/pmc > "$O/pmc_summary.md" && cut -c1-200 "$O/pmc_summary.md"
