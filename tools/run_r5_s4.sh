#!/usr/bin/env bash
# round 5, session 4: the N = 8 RCCL rehearsal on one GPU (python bench.py --gpus 8, defaults)
set -eo pipefail
out=gpurun_out/r5_s4; mkdir -p $out
export DCCL_BENCH_RCCL_REHEARSAL=1
start=$(date +%s)
timeout -k 10 900 python -u bench.py --gpus 8 > $out/bench_n8_rehearsal.json 2> $out/bench_n8_rehearsal.err
echo "n8 rehearsal ok in $(( $(date +%s) - start )) s"
