#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, kernel tuning table, bench line, rocprof summary.
# Every GPU step has its own time limit; steps are chained so the first failure ends the run.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${TAG:-r1}
mkdir -p "$out"
export TMPDIR=/tmp
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1 || { tail -50 "$out/pytest_gpu.log"; exit 1; }
tail -3 "$out/pytest_gpu.log"
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 && cat "$out/smoke.log"
echo "== tune"; timeout -k 10 600 python tools/tune_reduce.py --out "$out/tune.json" > "$out/tune.log" 2>&1 && head -40 "$out/tune.json"
echo "== bench"; timeout -k 10 600 python bench.py > "$out/bench.json" 2> "$out/bench.err" && cat "$out/bench.json"
echo "== rocprof"; timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out/prof" -o bench --output-format csv -- python3 bench.py --steps 20 --no-cpu --no-host-staged > "$out/prof.log" 2>&1 && find "$out/prof" -name "*stats*" | head
