#!/usr/bin/env bash
# round 5, session 3: IPC tests after the token-read change, the scratch-allocation probe, the N = 8 RCCL
# rehearsal on one GPU (the driver's 8-GPU path: python bench.py --gpus 8, defaults)
set -eo pipefail
out=gpurun_out/r5_s3; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_direct.py tests/test_failures.py tests/test_c1_processes.py -m gpu -x -q \
   --timeout 240 --timeout-method thread -p no:cacheprovider > $out/pytest_ipc.log 2>&1
echo "ipc tests ok"
timeout -k 10 400 python -u tools/scratch_vmm.py --rounds 5 --out $out/scratch_vmm.json > $out/scratch_vmm.log 2>&1
echo "vmm ok"
export DCCL_BENCH_RCCL_REHEARSAL=1
start=$(date +%s)
timeout -k 10 900 python -u bench.py --gpus 8 > $out/bench_n8_rehearsal.json 2> $out/bench_n8_rehearsal.err
echo "n8 rehearsal ok in $(( $(date +%s) - start )) s"
