#!/bin/bash
# One parameterised GPU-box runner (replaces the per-session scripts of round 1).
#
#   gpurun -- bash scripts/gpu.sh STEP [STEP ...]
#
# Steps (each runs under its own time limit; the first failure ends the call):
#   build      rebuild the HIP library in-tree if stale (sources newer than the .so)
#   tests      pytest -m gpu (all GPU tests, one process)
#   kernels    pytest tests/test_kernels_gpu.py only
#   smoke      __graft_entry__.smoke()
#   bench      bench.py --steps 50 --warmup 10 (JSON -> gpurun_out/bench.json)
#   eager      bench.py --engine eager (same-box PyTorch eager baseline)
#   prof       rocprofv3 --kernel-trace --stats of bench.py (summary -> gpurun_out/prof_summary.txt)
#   pmc        three rocprofv3 --pmc passes over scripts/prof_step_kernels.py
#   lab        scripts/gemm_lab.py (LAB_ARGS env passes flags)
#   py:FILE    python -u FILE (PY_ARGS env passes flags), e.g. py:scripts/kernel_bench.py
#   ab         alternating A/B of command-line variants: AB_CMD (a python command line printing one
#              JSON line), AB_VALUES ('|'-separated extra flags, one set per variant), AB_ROUNDS
#              (default 2); run i of variant v appends to gpurun_out/ab/v<v>.jsonl, then a summary.
#              e.g. AB_CMD="scripts/bench_configs.py topk --steps 40" AB_VALUES="--sparse-k 0|--sparse-k auto"
#   ktest:K    pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -k K
#   pytest:FILE[::K]  one GPU test file (optionally -k K)
#   profile:CMD  rocprofv3 --kernel-trace --stats of "python3 CMD" (top-20 summary)
# Extra bench flags: BENCH_ARGS env.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out"

run_step() {
  local s="$1"
  echo "=== step $s ($(date +%T))"
  case "$s" in
    build)
      timeout -k 10 300 python -m sparse_coding__amd.ops.build > "$O/build.log" 2>&1 || { tail -30 "$O/build.log"; return 1; } ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gputests.log" 2>&1
      local rc=$?; tail -25 "$O/gputests.log"; return $rc ;;
    kernels)
      timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > "$O/kernels.log" 2>&1
      local rc=$?; tail -25 "$O/kernels.log"; return $rc ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; local rc=$?; cat "$O/smoke.log"; return $rc ;;
    bench)
      timeout -k 10 400 python bench.py --steps 50 --warmup 10 ${BENCH_ARGS} > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; return 1; }
      cat "$O/bench.json" ;;
    eager)
      timeout -k 10 400 python bench.py --engine eager --steps 20 --warmup 5 --no-eval ${BENCH_ARGS} > "$O/bench_eager.json" 2> "$O/bench_eager.err" || { tail -20 "$O/bench_eager.err"; return 1; }
      cat "$O/bench_eager.json" ;;
    prof)
      rm -rf "$O/prof"
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 30 --warmup 5 --no-eval ${BENCH_ARGS} > "$O/prof.log" 2>&1) || { tail -20 "$O/prof.log"; return 1; }
      python3 - > "$O/prof_summary.txt" <<'PY' || return 1
import csv, glob
f = glob.glob("gpurun_out/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:20]:
    print(f"{r['Name'][:90]:90s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us {float(r['Percentage']):6.2f}%")
PY
      cat "$O/prof_summary.txt" ;;
    pmc)
      mkdir -p "$O/pmc"
      local S="$R/scripts/prof_step_kernels.py"
      (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d "$O/pmc/p1" -o p1 --output-format csv -- python3 "$S" > "$O/pmc/p1.log" 2>&1) || { tail -20 "$O/pmc/p1.log"; return 1; }
      (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM -d "$O/pmc/p2" -o p2 --output-format csv -- python3 "$S" > "$O/pmc/p2.log" 2>&1) || { tail -20 "$O/pmc/p2.log"; return 1; }
      (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d "$O/pmc/p3" -o p3 --output-format csv -- python3 "$S" > "$O/pmc/p3.log" 2>&1) || { tail -20 "$O/pmc/p3.log"; return 1; }
      python3 scripts/pmc_summary.py gpurun_out/pmc > "$O/pmc_summary.md" && cat "$O/pmc_summary.md" ;;
    lab)
      timeout -k 10 400 python -u scripts/gemm_lab.py ${LAB_ARGS} > "$O/gemm_lab.log" 2>&1; local rc=$?; cat "$O/gemm_lab.log"; return $rc ;;
    ab)
      mkdir -p "$O/ab"
      local IFS_OLD="$IFS"; IFS='|' read -r -a variants <<< "${AB_VALUES}"; IFS="$IFS_OLD"
      for r in $(seq 1 "${AB_ROUNDS:-2}"); do
        for i in "${!variants[@]}"; do
          timeout -k 10 300 python ${AB_CMD} ${variants[$i]} >> "$O/ab/v$i.jsonl" 2>> "$O/ab/err.log" || { tail -20 "$O/ab/err.log"; return 1; }
        done
      done
      grep -o '"ms_per_step": [0-9.]*\|"solve_ms_all_models": [0-9.]*' "$O"/ab/*.jsonl ;;
    pytest:*)
      # pytest:FILE[::K] -- one GPU test file (optionally -k K), one process
      local spec="${s#pytest:}" f k=""
      f="${spec%%::*}"; [[ "$spec" == *::* ]] && k="${spec#*::}"
      timeout -k 10 900 python -u -m pytest "$f" -m gpu -x -v --timeout 300 --timeout-method thread ${k:+-k "$k"} > "$O/pytest_$(basename "$f" .py).log" 2>&1
      local rc=$?; tail -15 "$O/pytest_$(basename "$f" .py).log"; return $rc ;;
    ktest:*)
      timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -x -q --timeout 300 --timeout-method thread -k "${s#ktest:}" > "$O/ktest.log" 2>&1
      local rc=$?; tail -15 "$O/ktest.log"; return $rc ;;
    profile:*)
      rm -rf "$O/profile"
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/profile" -o run --output-format csv -- python3 $R/${s#profile:} > "$O/profile.log" 2>&1) || { tail -20 "$O/profile.log"; return 1; }
      python3 - > "$O/profile_summary.txt" <<'PY' || return 1
import csv, glob
f = glob.glob("gpurun_out/profile/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:20]:
    print(f"{r['Name'][:90]:90s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us {float(r['Percentage']):6.2f}%")
PY
      cat "$O/profile_summary.txt" ;;
    py:*)
      local f="${s#py:}"
      timeout -k 10 600 python -u "$f" ${PY_ARGS} > "$O/$(basename "$f" .py).log" 2>&1; local rc=$?
      tail -40 "$O/$(basename "$f" .py).log"; return $rc ;;
    *)
      echo "unknown step $s"; return 2 ;;
  esac
}

for s in "$@"; do
  run_step "$s" || { echo "=== step $s FAILED"; exit 1; }
done
echo "=== all steps ok"
