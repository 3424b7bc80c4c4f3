#!/usr/bin/env bash
# round 5, session 8: second-box evidence for the kept size-row cells and the mid-size window form: the 1 GiB
# row everywhere (libdccl_p1, A) against the shipped table (B) at 16 / 32 / 64 MiB
set -eo pipefail
out=gpurun_out/r5_s8; mkdir -p $out
STEMS="multi,chain,multi_strad,chain_strad,multi_src+4,chain_src+4,multi_dst+2_src+4,chain_dst+2_src+4"
for mib in 16 32 64; do
  timeout -k 10 300 python -u tools/ab_cases.py dccl_amd/lib_ab/libdccl_p1.so dccl_amd/lib/libdccl_amd.so \
     --all-k "$STEMS" --mib $mib --rounds 7 --out $out/ab_kept_${mib}mib.json > $out/ab_kept_${mib}mib.log 2>&1
  echo "ab $mib"
done
