#!/usr/bin/env bash
# Build a second copy of the product library with extra compile flags, for tools/ab_combine.py
# (tuning only):  tools/build_ab.sh NAME "-DFLAG ..."  ->  dccl_amd/lib_ab/libdccl_NAME.so
set -euo pipefail
root="$(cd "$(dirname "$0")/.." && pwd)"
name="$1"; shift
flags="${1:-}"
out="$root/build/ab_$name"; mkdir -p "$out" "$root/dccl_amd/lib_ab"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
common=(-std=c++17 -O3 -fPIC -Wall -Wno-unused-command-line-argument -I"$root/include" -I"$root/dccl_amd/csrc" --offload-arch=gfx950)
pids=(); objs=()
for f in "$root"/dccl_amd/csrc/*.hip "$root"/dccl_amd/csrc/*.cpp; do
  o="$out/$(basename "$f").o"; objs+=("$o")
  x=(); [[ "$f" == *.hip ]] && x=(-x hip)
  # shellcheck disable=SC2086
  "$HIPCC" "${x[@]}" "${common[@]}" $flags -c "$f" -o "$o" & pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
"$HIPCC" --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "$root/dccl_amd/lib_ab/libdccl_$name.so"
echo "$root/dccl_amd/lib_ab/libdccl_$name.so"
