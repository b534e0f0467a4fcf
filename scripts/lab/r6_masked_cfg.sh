# masked config: encoder / code-gradient GEMM configurations (SC_GEMM_CFG epi:cfg), masked and unmasked ms
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_mcfg; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for spec in def "0:9,7:9" "0:25,7:25" "0:13,7:13" "0:1,7:1"; do
    if [ "$spec" = def ]; then e=""; else e=$spec; fi
    tag=$(echo $spec | tr ':,' '_-')
    SC_GEMM_CFG=$e timeout -k 10 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/m_$tag.jsonl 2>> $O/err.log || exit 1
  done
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$O/m_*.jsonl')):
    rs=[json.loads(l) for l in open(f)]
    print(f.split('/')[-1], [(r['masked_ms_per_step'], r['unmasked_ms_per_step'], r['time_ratio']) for r in rs])"
