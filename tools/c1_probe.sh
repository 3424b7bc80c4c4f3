set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/c1probe; mkdir -p $out
cli=dccl_amd/bin/dccl_cli
for algo in ring direct rabenseifner; do
 for g in -1 0; do
  echo "== $algo g=$g"
  DCCL_ALLREDUCE_ALGORITHM=$algo timeout -k 5 120 $cli -a all_reduce -t float32 -c 1024 -r 1000 -w 10 -n 4 -g $g | python3 -c "import sys,json; r=[json.loads(l) for l in sys.stdin if l.startswith('{')]; print(max(x['us_per_call'] for x in r), r[0]['first'], set(x['rc'] for x in r))"
 done
done
echo "== ring device, 2 ranks"
timeout -k 5 120 $cli -a all_reduce -t float32 -c 1024 -r 1000 -w 10 -n 2 -g 0 | python3 -c "import sys,json; r=[json.loads(l) for l in sys.stdin if l.startswith('{')]; print(max(x['us_per_call'] for x in r))"
echo "== ring device world 1"
timeout -k 5 120 $cli -a all_reduce -t float32 -c 1024 -r 1000 -w 10 -n 1 -g 0 | python3 -c "import sys,json; r=[json.loads(l) for l in sys.stdin if l.startswith('{')]; print(max(x['us_per_call'] for x in r))"
cd /tmp && export TMPDIR=/tmp
timeout -k 5 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_ring -o ring --output-format csv -- $GRAFT_REPO_ROOT/$cli -a all_reduce -t float32 -c 1024 -r 200 -w 10 -n 4 -g 0 > /dev/null
DCCL_ALLREDUCE_ALGORITHM=direct timeout -k 5 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_direct -o direct --output-format csv -- $GRAFT_REPO_ROOT/$cli -a all_reduce -t float32 -c 1024 -r 200 -w 10 -n 4 -g 0 > /dev/null
echo done
