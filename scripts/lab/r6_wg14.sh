# headline weight gradients (epi 3, layout 0) on the eight-wave 256x128 block (cfg 14) vs 256x256
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_wg14; rm -rf $O; mkdir -p $O
true

for r in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/def.jsonl 2>> $O/err.log || exit 1
  SC_GEMM_CFG=3/0:14 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/wg14.jsonl 2>> $O/err.log || exit 1
done
python3 -c "
import json
for v in ('def','wg14'): print(v, [json.loads(l)['ms_per_step'] for l in open('$O/'+v+'.jsonl')])"
