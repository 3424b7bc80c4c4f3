#!/usr/bin/env bash
# rocprofv3 passes over tools/misaligned_probe.py (misaligned-recv combine): kernel trace, FETCH_SIZE, WRITE_SIZE,
# TCC EA request sizes.  OUT sets the output directory; PROBE_ARGS are passed to the probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; out=${OUT:-gpurun_out/r2/s5}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/kt -o m --output-format csv -- python3 tools/misaligned_probe.py ${PROBE_ARGS:-} > $out/kt.log 2>&1; echo kt rc=$?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/f -o m -- python3 tools/misaligned_probe.py ${PROBE_ARGS:-} > $out/f.log 2>&1; echo f rc=$?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/w -o m -- python3 tools/misaligned_probe.py ${PROBE_ARGS:-} > $out/w.log 2>&1; echo w rc=$?
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_WRREQ_64B --kernel-trace --output-format csv -d $out/q -o m -- python3 tools/misaligned_probe.py ${PROBE_ARGS:-} > $out/q.log 2>&1; echo q rc=$?
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ TCC_EA0_WRREQ_64B --kernel-trace --output-format csv -d $out/wq -o m -- python3 tools/misaligned_probe.py ${PROBE_ARGS:-} > $out/wq.log 2>&1; echo wq rc=$?
