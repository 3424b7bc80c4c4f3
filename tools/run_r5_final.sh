#!/usr/bin/env bash
# round 5 final-tree validation: the full GPU suite, smoke(), and the bench line as the driver runs it
set -eo pipefail
out=gpurun_out/r5_final; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
   > $out/pytest_gpu.log 2>&1
echo "pytest ok"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
echo "smoke ok"
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err
echo "bench ok"
