set -o pipefail
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r2/s5; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/kt -o m --output-format csv -- python3 tools/misaligned_probe.py > $out/kt.log 2>&1; echo kt rc=$?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/f -o m -- python3 tools/misaligned_probe.py > $out/f.log 2>&1; echo f rc=$?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/w -o m -- python3 tools/misaligned_probe.py > $out/w.log 2>&1; echo w rc=$?
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_WRREQ_64B --kernel-trace --output-format csv -d $out/q -o m -- python3 tools/misaligned_probe.py > $out/q.log 2>&1; echo q rc=$?
