#!/usr/bin/env bash
# FETCH_SIZE and WRITE_SIZE passes (separate: they do not fit one pass on gfx950) over tools/issue_probe.py's
# cases (ONLY = comma list), each under its own hard limit; the summary joins every dispatch with its counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
out=gpurun_out/r3/${TAG:-traffic}; mkdir -p "$out/fetch" "$out/write"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$out/fetch" -o p -- python3 tools/issue_probe.py --launches 3 ${ONLY:+--only "$ONLY"} > "$out/fetch/run.log" 2>&1; rc=$?; echo "fetch rc=$rc"
[[ $rc -ne 0 ]] && exit $rc
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$out/write" -o p -- python3 tools/issue_probe.py --launches 3 ${ONLY:+--only "$ONLY"} > "$out/write/run.log" 2>&1; rc=$?; echo "write rc=$rc"
[[ $rc -ne 0 ]] && exit $rc
python3 tools/issue_probe.py --parse "$out" --out "$out/summary.json" > /dev/null 2>&1; echo "parse rc=$?"
