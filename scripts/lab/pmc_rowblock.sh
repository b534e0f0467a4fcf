set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/pmc_rb"
mkdir -p "$O"
B="$GRAFT_REPO_ROOT/scripts/lab/rowblock_stamps"
(cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d "$O/p1" -o p1 --output-format csv -- "$B" > "$O/p1.log" 2>&1) || { tail -20 "$O/p1.log"; exit 1; }
(cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM -d "$O/p2" -o p2 --output-format csv -- "$B" > "$O/p2.log" 2>&1) || { tail -20 "$O/p2.log"; exit 1; }
(cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d "$O/p3" -o p3 --output-format csv -- "$B" > "$O/p3.log" 2>&1) || { tail -20 "$O/p3.log"; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_rb > "$O/summary.md"; grep -i "rowblock\|kernel" "$O/summary.md" | cut -c1-400 | head -20
