set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/algo; mkdir -p $out
cli=dccl_amd/bin/dccl_cli
for n in 2 4 8; do
 for c in 1024 262144 4194304 16777216; do
  for algo in ring direct; do
   r=200; [ $c -ge 4194304 ] && r=30
   us=$(DCCL_ALLREDUCE_ALGORITHM=$algo timeout -k 5 120 $cli -a all_reduce -t float32 -c $((c / n * n)) -r $r -w 5 -n $n -g 0 | python3 -c "import sys,json; r=[json.loads(l) for l in sys.stdin if l.startswith('{')]; print(max(x['us_per_call'] for x in r))")
   echo "{\"world\": $n, \"count\": $c, \"algo\": \"$algo\", \"us\": $us}" | tee -a $out/algo.jsonl
  done
 done
done
