#!/usr/bin/env bash
# Host-buffer all_reduce through dccl_cli (4 thread-ranks, fp32 Sum): ring vs the direct default, small to
# large counts; µs per call, max over ranks.  Output: gpurun_out/hostar/host_ar.jsonl
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/hostar; mkdir -p $out; : > $out/host_ar.jsonl
for c in 1024 1048576 16777216 67108864; do
  for algo in ring auto; do
    r=200; [ $c -ge 16777216 ] && r=5
    us=$(DCCL_ALLREDUCE_ALGORITHM=$algo timeout -k 5 300 dccl_amd/bin/dccl_cli -a all_reduce -t float32 -c $c -r $r -w 2 -n 4 -g -1 | python3 -c "import sys,json; r=[json.loads(l) for l in sys.stdin if l.startswith('{')]; print(max(x['us_per_call'] for x in r))")
    echo "{\"count\": $c, \"algo\": \"$algo\", \"us\": $us}" | tee -a $out/host_ar.jsonl
  done
done
