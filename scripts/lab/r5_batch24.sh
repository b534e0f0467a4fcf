#!/bin/bash
# round 5, GPU batch 24: PMC of the headline step's kernels IN SEQUENCE (eager step loop), to compare
# with batch 18's kernels-on-their-own view
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b24
mkdir -p $O
S="$R/scripts/lab/prof_step_eager.py"
python -c "from sparse_coding__amd.ops import build as b; b.build(force=False)" || exit 1
timeout -k 10 300 python "$S" > $O/dry.log 2>&1 || { tail -20 $O/dry.log; exit 1; }
(cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$O/trace" -o tr --output-format csv -- python3 "$S" > "$O/trace.log" 2>&1) || { tail -20 "$O/trace.log"; exit 1; }
(cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d "$O/pmc/p1" -o p1 --output-format csv -- python3 "$S" > "$O/p1.log" 2>&1) || { tail -20 "$O/p1.log"; exit 1; }
(cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM -d "$O/pmc/p2" -o p2 --output-format csv -- python3 "$S" > "$O/p2.log" 2>&1) || { tail -20 "$O/p2.log"; exit 1; }
(cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d "$O/pmc/p3" -o p3 --output-format csv -- python3 "$S" > "$O/p3.log" 2>&1) || { tail -20 "$O/p3.log"; exit 1; }
(cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE -d "$O/pmc/p4" -o p4 --output-format csv -- python3 "$S" > "$O/p4.log" 2>&1) || { tail -20 "$O/p4.log"; exit 1; }
python3 scripts/pmc_summary.py $O/pmc > "$O/pmc_summary.md" && cut -c1-200 "$O/pmc_summary.md"
python3 scripts/lab/step_budget.py $O/trace 120 > $O/step_budget.txt; cat $O/step_budget.txt
