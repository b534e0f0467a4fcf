# Masked decoder K pipeline: BK64 x 2 (default) vs BK32 x 5 (cfg 5) vs pipelined BK32 x 5 (cfg 21)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_mdec; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_masked_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for c in def 1:5 1:21; do
    if [ $c = def ]; then e=""; else e=$c; fi
    SC_GEMM_CFG=$e timeout -k 10 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/m_${c/:/_}.jsonl 2>> $O/err.log || exit 1
  done
done
python3 -c "
import json
for v in ('def','1_5','1_21'):
    rs=[json.loads(l) for l in open('$O/m_'+v+'.jsonl')]
    print(v, [(r['masked_ms_per_step'], r['unmasked_ms_per_step'], r['time_ratio']) for r in rs])"
