#!/bin/bash
# Kernel traces of the driver's short bench (20/5) under the new and the round-3 harness and of a
# long run; per-step timelines of each run's last 20 steps.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/timeline_ab
mkdir -p $O
T="timeout -k 10 240"
$T rocprofv3 --kernel-trace -d $O/new20 -- python3 bench.py --steps 20 --warmup 5 --no-eval > $O/new20.json 2> $O/new20.err
$T rocprofv3 --kernel-trace -d $O/old20 -- python3 scripts/lab/bench_r3_harness.py --steps 20 --warmup 5 --no-eval > $O/old20.json 2> $O/old20.err
$T rocprofv3 --kernel-trace -d $O/new200 -- python3 bench.py --steps 200 --warmup 20 --no-eval > $O/new200.json 2> $O/new200.err
for r in new20 old20 new200; do python3 scripts/lab/step_timeline.py $O/$r 20 > $O/$r.timeline.jsonl; tail -1 $O/$r.timeline.jsonl; done
# ensemble sharding through one RCCL rank (multi-step groups: per-step batch all-gathers + one replay per group)
$T python3 bench.py --steps 200 --warmup 20 --no-eval --force-dist --parallelism es --compare-parallelism 0 > $O/es1_200.json 2> $O/es1_200.err
$T python3 bench.py --steps 20 --warmup 5 --no-eval --force-dist --parallelism es --compare-parallelism 0 > $O/es1_20.json 2> $O/es1_20.err
for r in es1_200 es1_20; do python3 -c "import json,sys; d=json.loads(open('$O/$r.json').read().strip().splitlines()[-1]); print('$r', d['ms_per_step'], d['config']['parallelism'])"; done
