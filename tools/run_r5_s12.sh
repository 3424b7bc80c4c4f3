#!/usr/bin/env bash
set -eo pipefail
out=gpurun_out/r5_s12; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_bench_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread \
   -p no:cacheprovider > $out/pytest_bench.log 2>&1
echo "bench tests ok"
export DCCL_BENCH_RCCL_REHEARSAL=1
start=$(date +%s)
timeout -k 10 900 python -u bench.py --gpus 8 > $out/bench_n8_rehearsal.json 2> $out/bench_n8_rehearsal.err
echo "n8 rehearsal ok in $(( $(date +%s) - start )) s"
