# A/B: ab_old/ (a HEAD copy built in-tree) vs this tree, interleaved bench runs on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_ab; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_headline_grad_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3 4; do
  (cd ab_old && timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval) >> $O/old.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/new.jsonl 2>> $O/err.log || exit 1
done
python3 -c "
import json
for v in ('old','new'): print(v, [json.loads(l)['ms_per_step'] for l in open('$O/'+v+'.jsonl')])"
