#!/usr/bin/env bash
# round 5: the headline alone (bench.py's timed region, PMC traffic, CPU baseline skipped), for the per-box spread
set -eo pipefail
out=gpurun_out/r5_headline; mkdir -p $out
tag=$(date +%s)
timeout -k 10 400 python -u bench.py --no-configs --no-host-staged --no-cpu --no-other-layout \
   > $out/bench_$tag.json 2> $out/bench_$tag.err
echo "headline ok"
