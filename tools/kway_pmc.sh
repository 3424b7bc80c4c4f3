#!/usr/bin/env bash
# FETCH_SIZE and WRITE_SIZE passes over tools/kway_pmc_probe.py (k-way and chain, k = 1..8), sources at
# byte offset PHASE (default 4: the phased kernels); each pass under its own hard time limit.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
kout=gpurun_out/${TAG:-r2}/kway_pmc_phase${PHASE:-4}
mkdir -p "$kout/fetch" "$kout/write"
export TMPDIR=/tmp
echo "== FETCH_SIZE"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$kout/fetch" -o p -- \
  python3 tools/kway_pmc_probe.py --phase "${PHASE:-4}" > "$kout/fetch/run.log" 2>&1
echo "== WRITE_SIZE"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$kout/write" -o p -- \
  python3 tools/kway_pmc_probe.py --phase "${PHASE:-4}" > "$kout/write/run.log" 2>&1
python3 tools/kway_pmc_probe.py --parse "$kout" --out "$kout/summary.json" > "$kout/parse.log" 2>&1
echo "== done"
