#!/usr/bin/env bash
# round 5, session 7: the new own-only-off-phase chain test, then the IPC churn stress of the (only) scratch path
set -eo pipefail
out=gpurun_out/r5_s7; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "own_only or windows_tuned" \
   --timeout 240 --timeout-method thread -p no:cacheprovider > $out/pytest_chain.log 2>&1
echo "chain tests ok"
timeout -k 10 700 python -u tools/ipc_churn_stress.py --runs 12 --world 4 --mib 1 --rounds 100 --register \
   > $out/churn_w4_reg.json 2> $out/churn_w4_reg.err
echo "churn w4 ok"
timeout -k 10 400 python -u tools/ipc_churn_stress.py --runs 12 --world 2 --mib 1 --rounds 140 \
   > $out/churn_w2.json 2> $out/churn_w2.err
echo "churn w2 ok"
