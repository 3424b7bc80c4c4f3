#!/usr/bin/env bash
# One GPU-box session of round 3: the whole -m gpu suite (failures reported, not fatal), smoke, the bench line,
# and optionally the issue-side PMC passes of tools/issue_probe.py (ISSUE=1) and a rocprof kernel trace of the
# bench (PROF=1).  A step that times out or crashes (status 124 or above 128) ends the session: nothing more
# runs on the GPU after it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r3/${TAG:-s1}; mkdir -p "$out"; export TMPDIR=/tmp
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
  tail -c 3000 "$out/bench.json"; echo
  stop_if_fatal $rc
fi
if [[ -n "${ISSUE:-}" ]]; then
  echo "== counter list"
  timeout -s KILL 90 rocprofv3 -L > "$out/counters.txt" 2>&1; echo "L rc=$?"
  pass_no=0
  for want in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM" \
              "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM" \
              "TA_TA_BUSY TA_BUFFER_READ_WAVEFRONTS TD_TD_BUSY TD_TC_STALL TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY"; do
    pass_no=$((pass_no + 1))
    have=""; for c in $want; do grep -qw "$c" "$out/counters.txt" && have="$have $c"; done
    echo "pass $pass_no:$have"
    [[ -z "$have" ]] && continue
    mkdir -p "$out/issue/p$pass_no"
    timeout -s KILL 240 rocprofv3 --pmc $have --kernel-trace --output-format csv -d "$out/issue/p$pass_no" -o p -- python3 tools/issue_probe.py ${ISSUE_ARGS:-} > "$out/issue/p$pass_no/run.log" 2>&1; rc=$?; echo "pass $pass_no rc=$rc"
    stop_if_fatal $rc
  done
  python3 tools/issue_probe.py --parse "$out/issue" --out "$out/issue_summary.json" > /dev/null 2>&1; echo "parse rc=$?"
fi
if [[ -n "${PROF:-}" ]]; then
  echo "== rocprof kernel trace"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out/prof" -o bench --output-format csv -- python3 bench.py --steps 50 --no-cpu --no-host-staged --no-other-layout --no-pmc --no-configs --c5-gib 0 > "$out/prof.log" 2>&1; rc=$?; echo "prof rc=$rc"
  stop_if_fatal $rc
fi
echo "== done"
