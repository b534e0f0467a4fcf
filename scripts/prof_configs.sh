#!/bin/bash
# Kernel-trace profiles of the non-headline configs (top-k, masked / unmasked, FISTA-in-loss),
# one rocprofv3 run each; summaries -> gpurun_out/prof_<name>.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out"
mkdir -p "$O"
run() {
  local name="$1"; shift
  rm -rf "$O/prof_$name"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$name" -o run --output-format csv -- python3 "$R/scripts/bench_configs.py" "$@" > "$O/prof_$name.log" 2>&1) || { tail -20 "$O/prof_$name.log"; return 1; }
  python3 "$R/scripts/prof_summary.py" "$O/prof_$name" > "$O/prof_$name.txt" && echo "== $name" && cat "$O/prof_$name.txt"
}
for spec in "$@"; do
  case "$spec" in
    topk) run topk topk --steps 20 --warmup 3 ;;
    masked) run masked masked --variant masked --steps 50 --warmup 5 ;;
    unmasked) run unmasked masked --variant unmasked --steps 50 --warmup 5 ;;
    fistaloss) run fistaloss fistaloss --steps 10 --warmup 2 --iters 50 ;;
    *) echo "unknown $spec"; exit 2 ;;
  esac || exit 1
done
