#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, bench line, rocprof kernel-trace summary, two PMC
# passes (FETCH_SIZE, WRITE_SIZE: separate runs), the secondary suite.  Every GPU step has its
# own time limit and the steps are chained, so the first failure ends the run.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${TAG:-r2}
mkdir -p "$out"
export TMPDIR=/tmp
if [[ -z "${SKIP_TESTS:-}" ]]; then
echo "== pytest -m gpu"
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1 || { tail -60 "$out/pytest_gpu.log"; exit 1; }
tail -3 "$out/pytest_gpu.log"
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
cat "$out/smoke.log"
fi
echo "== bench"
timeout -k 10 600 python bench.py > "$out/bench.json" 2> "$out/bench.err"
cat "$out/bench.json"
if [[ "${PROF:-1}" != 0 ]]; then
  echo "== rocprof kernel trace"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out/prof" -o bench --output-format csv -- python3 bench.py --steps 50 --no-cpu --no-host-staged --no-other-layout --no-pmc --no-configs --c5-gib 0 > "$out/prof.log" 2>&1
  echo "== pmc FETCH_SIZE"
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o fetch -- python3 tools/pmc_probe.py > "$out/pmc_fetch.log" 2>&1
  echo "== pmc WRITE_SIZE"
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o write -- python3 tools/pmc_probe.py > "$out/pmc_write.log" 2>&1
fi
if [[ -n "${KWAYW:-}" ]]; then
  echo "== k-way / chain occupancy caps at 1 GiB"
  timeout -k 10 600 python tools/kway_waves.py --out "$out/kway_waves.json" > "$out/kway_waves.log" 2>&1
  tail -20 "$out/kway_waves.log"
fi
if [[ -n "${CEILING:-}" ]]; then
  echo "== HBM ceiling probes"
  timeout -k 10 300 python tools/ceiling_probe.py --out "$out/ceiling.json" > "$out/ceiling.log" 2>&1
  cat "$out/ceiling.log"
fi
if [[ -n "${SUITE:-}" ]]; then
  echo "== suite ($SUITE)"
  timeout -k 10 900 python tools/bench_suite.py --parts "$SUITE" --out "$out/suite.json" > "$out/suite.log" 2>&1
  tail -30 "$out/suite.log"
fi
if [[ -n "${SUITE_STAGED:-}" ]]; then
  echo "== host path with zero-copy disabled"
  DCCL_HOST_ZEROCOPY_MAX=0 timeout -k 10 600 python tools/bench_suite.py --parts host,c1 --out "$out/suite_nozc.json" > "$out/suite_nozc.log" 2>&1
  tail -20 "$out/suite_nozc.log"
fi
echo "== done"
