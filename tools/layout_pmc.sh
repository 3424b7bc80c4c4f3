#!/usr/bin/env bash
# PMC passes over fast and slow operand placements (tools/layout_pmc_probe.py); one counter group per
# rocprofv3 run (at most 4 TCC counters each), every run under its own hard time limit.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${TAG:-r2}/layout_pmc
mkdir -p "$out"
export TMPDIR=/tmp
passes=(
  "TCC_EA0_RDREQ TCC_EA0_RDREQ_LEVEL TCC_EA0_WRREQ TCC_EA0_WRREQ_LEVEL"
  "TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_TOO_MANY_EA_WRREQS_STALL TCC_TAG_STALL"
  "TCC_EA0_RDREQ_GMI_32B TCC_EA0_RDREQ_DRAM TCC_EA0_WRREQ_WRITE_GMI_32B TCC_EA0_WRREQ_DRAM"
  "TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_WRREQ_64B"
)
i=0
for p in "${passes[@]}"; do
  d="$out/p$i"
  mkdir -p "$d"
  echo "== pass $i: $p"
  # shellcheck disable=SC2086
  timeout -s KILL 180 rocprofv3 --pmc $p --kernel-trace --output-format csv -d "$d" -o p -- \
    python3 tools/layout_pmc_probe.py --pairs "${PAIRS:-8}" > "$d/run.log" 2>&1
  i=$((i + 1))
done
python3 tools/layout_pmc_probe.py --parse "$out" --out "$out/summary.json" > "$out/parse.log" 2>&1 || echo "layout parse failed"

if [[ -n "${KWAY:-}" ]]; then
  kout=gpurun_out/${TAG:-r2}/kway_pmc
  mkdir -p "$kout/fetch" "$kout/write"
  echo "== k-way FETCH_SIZE"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$kout/fetch" -o p -- \
    python3 tools/kway_pmc_probe.py > "$kout/fetch/run.log" 2>&1
  echo "== k-way WRITE_SIZE"
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$kout/write" -o p -- \
    python3 tools/kway_pmc_probe.py > "$kout/write/run.log" 2>&1
  python3 tools/kway_pmc_probe.py --parse "$kout" --out "$kout/summary.json" > "$kout/parse.log" 2>&1 || echo "kway parse failed"
  echo "== k-way done"
fi
echo "== all done"
