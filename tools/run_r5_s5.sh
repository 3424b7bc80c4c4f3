#!/usr/bin/env bash
# round 5, session 5: the N = 1 bench at the final tree (as the driver runs it), then the same command under
# rocprofv3 --kernel-trace --stats (PMC passes off: no profiler inside the profiler) and the headline split
set -eo pipefail
out=gpurun_out/r5_s5; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err
echo "bench ok"
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 -u bench.py --no-pmc \
   > $out/bench_profiled.json 2> $out/bench_profiled.err
echo "profiled ok"
python tools/rocprof_headline.py $out/prof > $out/rocprof_headline_split.json
echo "split ok"
