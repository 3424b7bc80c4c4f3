#!/usr/bin/env bash
# round-5 caps pruning A/B: round-4 library (A) against the pruned table (B) at 16/32/64/1024 MiB
set -eo pipefail
mkdir -p gpurun_out/r5_ab
STEMS="multi,chain,multi_strad,chain_strad,multi_src+4,chain_src+4,multi_dst+2,chain_dst+2,multi_dst+2_src+4,chain_dst+2_src+4"
for mib in 16 32 64 1024; do
  timeout -k 10 300 python -u tools/ab_cases.py dccl_amd/lib_ab/libdccl_r4.so dccl_amd/lib_ab/libdccl_p1.so \
     --cases pair,pair_src+4,pair_dst+1 --all-k "$STEMS" --mib $mib --rounds 5 --out gpurun_out/r5_ab/ab_p1_${mib}mib.json \
     > gpurun_out/r5_ab/ab_p1_${mib}mib.log 2>&1
  echo "done $mib"
done
