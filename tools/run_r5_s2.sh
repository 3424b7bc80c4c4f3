#!/usr/bin/env bash
# round 5, session 2: GPU suite at the pruned tree, then the caps A/B (round-4 library vs this one) and the
# scratch-allocation probe
set -eo pipefail
out=gpurun_out/r5_s2; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
   > $out/pytest_gpu.log 2>&1
echo "pytest ok"
STEMS="multi,chain,multi_strad,chain_strad,multi_src+4,chain_src+4,multi_dst+2,chain_dst+2,multi_dst+2_src+4,chain_dst+2_src+4"
for mib in 16 32 64 1024; do
  timeout -k 10 300 python -u tools/ab_cases.py dccl_amd/lib_ab/libdccl_r4.so dccl_amd/lib/libdccl_amd.so \
     --cases pair,pair_src+4,pair_dst+1 --all-k "$STEMS" --mib $mib --rounds 5 --out $out/ab_final_${mib}mib.json \
     > $out/ab_final_${mib}mib.log 2>&1
  echo "ab $mib"
done
timeout -k 10 400 python -u tools/scratch_vmm.py --rounds 5 --out $out/scratch_vmm.json > $out/scratch_vmm.log 2>&1
echo "vmm ok"
