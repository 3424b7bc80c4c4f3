#!/usr/bin/env bash
# Round 3: the misaligned-destination forms and caps (tools/unaligned_forms_probe.py), then the GPU tests of the
# misaligned classes and the failure paths.  A step that times out or crashes ends the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; out=gpurun_out/r3/${TAG:-s3}; mkdir -p $out
timeout -k 10 600 python tools/unaligned_forms_probe.py ${FORMS_ARGS:-} --out $out/forms.json > $out/forms.log 2> $out/forms.err; rc=$?; echo "forms rc=$rc"
[[ $rc -eq 124 || $rc -gt 128 ]] && exit $rc
[[ -n "${SKIP_TESTS:-}" ]] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "${PYTEST_K:-misaligned or unaligned or byte_offsets or alignment or failure or sticky or multi or chain}" > $out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest.log; grep -E "^(FAILED|ERROR)" $out/pytest.log | head || true
