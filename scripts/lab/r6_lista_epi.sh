set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_lepi; rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  SC_LISTA_EPI=0 timeout -k 10 200 python scripts/unrolled_bench.py --only-unrolled >> $O/off.jsonl 2>>$O/err.log || exit 1
  SC_LISTA_EPI=1 timeout -k 10 200 python scripts/unrolled_bench.py --only-unrolled >> $O/on.jsonl 2>>$O/err.log || exit 1
done
cat $O/off.jsonl $O/on.jsonl
