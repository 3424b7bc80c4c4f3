set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hwq
for q in 4 8 16; do
  for n in 4 8; do
    us=$(GPU_MAX_HW_QUEUES=$q DCCL_ALLREDUCE_ALGORITHM=ring timeout -k 5 120 dccl_amd/bin/dccl_cli -a all_reduce -t float32 -c 1024 -r 300 -w 5 -n $n -g 0 | python3 -c "import sys,json; r=[json.loads(l) for l in sys.stdin if l.startswith('{')]; print(max(x['us_per_call'] for x in r))")
    echo "{\"hw_queues\": $q, \"world\": $n, \"ring_us\": $us}" | tee -a gpurun_out/hwq/hwq.jsonl
  done
done
