# Decoder K pipeline: BK64 x 2 (cfg 1, default) vs BK32 x 5 (cfg 5) vs BK32 x 5 software-pipelined (cfg 21)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_dec; rm -rf $O; mkdir -p $O
true

PB_CFGS=1,5,21,13,29 PB_KERNELS=dec timeout -k 10 120 python scripts/pipe_bench.py > $O/pipe.jsonl 2>> $O/err.log || exit 1
cat $O/pipe.jsonl
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/c1.jsonl 2>> $O/err.log || exit 1
  SC_GEMM_CFG=1:5 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/c5.jsonl 2>> $O/err.log || exit 1
  SC_GEMM_CFG=1:21 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/c21.jsonl 2>> $O/err.log || exit 1
done
python3 -c "
import json
for v in ('c1','c5','c21'): print(v, [json.loads(l)['ms_per_step'] for l in open('$O/'+v+'.jsonl')])"
bash scripts/lab/r6_mdec.sh
