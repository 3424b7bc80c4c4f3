#!/usr/bin/env bash
# Round 3: A/B of two product builds on the alignment classes (tools/ab_cases.py), then the GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; out=gpurun_out/r3/${TAG:-ab}; mkdir -p $out
timeout -k 10 600 python tools/ab_cases.py ${AB_A:-dccl_amd/lib_ab/libdccl_r2.so} ${AB_B:-dccl_amd/lib/libdccl_amd.so} --rounds ${AB_ROUNDS:-5} ${AB_CASES:+--cases "$AB_CASES"} --out $out/ab.json > $out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat $out/ab.log
[[ $rc -eq 124 || $rc -gt 128 ]] && exit $rc
[[ -n "${SKIP_TESTS:-}" ]] && exit 0
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > $out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $out/pytest_gpu.log | head -20 || true
