set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_phases; rm -rf $O; mkdir -p $O/raw
timeout -k 10 120 scripts/lab/gemm_phases_128 $O/raw > $O/phases.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
python3 scripts/lab/phase_budget.py $O/raw 3 > $O/phase_budget.txt && cat $O/phase_budget.txt
