#!/usr/bin/env bash
# oracle/build_ref.sh — build the reference's CPU combine as a test oracle.
#
# Reads do_host_reduce<DT> straight from the read-only reference tree
# (/root/reference/src/core/internal_common.hpp:496-586) into a scratch directory
# OUTSIDE the repository, generates the one-line dccl/config.h the public header
# needs (CACHELINE_SIZE, /root/reference/config.h.in:2), and compiles
# oracle/ref_harness.cpp with the reference's Release flags
# (/root/reference/CMakeLists.txt:25).  The only output is
# oracle/_ref/libref_host_reduce.so (git-ignored; it travels to the GPU box so the
# bench can time the real reference loop).  No reference source enters the repo.
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
ref="${DCCL_REFERENCE:-/root/reference}"
hdr="$ref/src/core/internal_common.hpp"
if [[ ! -f "$hdr" || ! -f "$ref/include/dccl/dccl.hpp" ]]; then
    echo "build_ref: reference not present at $ref; skipping" >&2
    exit 0
fi
scratch="$(mktemp -d /tmp/dccl_ref_build.XXXXXX)"
trap 'rm -rf "$scratch"' EXIT
mkdir -p "$scratch/dccl" "$here/_ref"
echo '#define CACHELINE_SIZE 64' > "$scratch/dccl/config.h"
# Lines 496-586: `template<typename DT> ncclResult_t do_host_reduce(...) { ... }`.
sed -n '496,586p' "$hdr" > "$scratch/host_reduce_body.inc"
head -2 "$scratch/host_reduce_body.inc" | grep -q 'do_host_reduce' || {
    echo "build_ref: unexpected reference layout at $hdr:496" >&2; exit 1; }
g++ -std=c++17 -O3 -mprefer-vector-width=512 -fPIC -shared \
    -I"$ref/include" -I"$scratch" \
    "$here/ref_harness.cpp" -o "$here/_ref/libref_host_reduce.so"
# Benchmark-build variant (CMakeLists.txt:26): -Ofast -march=native.
g++ -std=c++17 -Ofast -march=native -mprefer-vector-width=512 -fPIC -shared \
    -I"$ref/include" -I"$scratch" \
    "$here/ref_harness.cpp" -o "$here/_ref/libref_host_reduce_native.so"
echo "build_ref: built $here/_ref/libref_host_reduce{,_native}.so"
