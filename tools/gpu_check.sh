#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, bench line, rocprof kernel-trace summary, two PMC
# passes (FETCH_SIZE, WRITE_SIZE: separate runs), the secondary suite.  Every GPU step has its
# own time limit and the steps are chained, so the first failure ends the run.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${TAG:-r1}
mkdir -p "$out"
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1 || { tail -60 "$out/pytest_gpu.log"; exit 1; }
tail -3 "$out/pytest_gpu.log"
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
cat "$out/smoke.log"
echo "== bench"
timeout -k 10 600 python bench.py > "$out/bench.json" 2> "$out/bench.err"
cat "$out/bench.json"
echo "== rocprof kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out/prof" -o bench --output-format csv -- python3 bench.py --steps 20 --no-cpu --no-host-staged > "$out/prof.log" 2>&1
echo "== pmc FETCH_SIZE"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o fetch -- python3 tools/pmc_probe.py > "$out/pmc_fetch.log" 2>&1
echo "== pmc WRITE_SIZE"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o write -- python3 tools/pmc_probe.py > "$out/pmc_write.log" 2>&1
if [[ -n "${SUITE:-1}" && "${SUITE:-1}" != 0 ]]; then
  echo "== suite"
  timeout -k 10 900 python tools/bench_suite.py --out "$out/suite.json" > "$out/suite.log" 2>&1
  tail -5 "$out/suite.log"
fi
echo "== done"
