#!/usr/bin/env bash
# One GPU-box session of round 2: the whole -m gpu suite (failures reported, not fatal), smoke, the bench
# line, and the k-way / chain occupancy sweep.  A step that times out or crashes (status 124, 134, 137,
# 139 or any signal) ends the session: nothing more runs on the GPU after it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r2/${TAG:-s1}; mkdir -p "$out"; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; if [[ $rc -eq 124 || $rc -gt 128 ]]; then echo "fatal rc=$rc: stopping"; exit "$rc"; fi; }
if [[ -z "${SKIP_TESTS:-}" ]]; then
  echo "== pytest"
  timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > "$out/pytest_gpu.log" 2>&1; rc=$?; echo "pytest rc=$rc"
  tail -3 "$out/pytest_gpu.log"; grep -E "^(FAILED|ERROR)" "$out/pytest_gpu.log" | head -20
  stop_if_fatal $rc
  echo "== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1; rc=$?; echo "smoke rc=$rc"
  stop_if_fatal $rc
fi
if [[ -z "${SKIP_BENCH:-}" ]]; then
  echo "== bench"
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$out/bench.json" 2> "$out/bench.err"; rc=$?; echo "bench rc=$rc"
  head -c 1500 "$out/bench.json"; echo
  stop_if_fatal $rc
fi
if [[ -n "${KWAYW:-}" ]]; then
  echo "== kway waves"
  timeout -k 10 600 python tools/kway_waves.py --out "$out/kway_waves.json" > "$out/kway_waves.log" 2>&1; rc=$?; echo "kway rc=$rc"
  stop_if_fatal $rc
fi
if [[ -n "${PROF:-}" ]]; then
  echo "== rocprof kernel trace"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out/prof" -o bench --output-format csv -- python3 bench.py --steps 50 --no-cpu --no-host-staged --no-other-layout --no-pmc --no-configs --c5-gib 0 > "$out/prof.log" 2>&1; rc=$?; echo "prof rc=$rc"
  stop_if_fatal $rc
fi
echo "== done"
