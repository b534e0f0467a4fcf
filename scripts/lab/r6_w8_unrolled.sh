# unrolled engines: their fp32 NT products (epi 3 layout 3) on the eight-wave 256x128 block (cfg 14)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_w8u; rm -rf $O; mkdir -p $O
SC_GEMM_CFG=3/3:14 timeout -k 10 300 python -u -m pytest tests/test_unrolled_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for m in "" "--residual"; do
    timeout -k 10 200 python scripts/unrolled_bench.py --only-unrolled $m >> $O/def.jsonl 2>> $O/err.log || exit 1
    SC_GEMM_CFG=3/3:14 timeout -k 10 200 python scripts/unrolled_bench.py --only-unrolled $m >> $O/w8.jsonl 2>> $O/err.log || exit 1
  done
done
cat $O/def.jsonl; echo; cat $O/w8.jsonl
