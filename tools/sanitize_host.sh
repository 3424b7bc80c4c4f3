#!/usr/bin/env bash
# Build the host-side C++ (transports, ring / direct algorithms, API, host staging, CLI) with a host
# sanitizer and drive the CPU-runnable collective paths (host buffers, no combine: all_gather,
# broadcast, world-size-1 all_reduce) through dccl_cli with 2-8 thread-ranks.
#   tools/sanitize_host.sh thread|address|undefined
# Device code is untouched (-Xarch_host): GPU sanitizers are not used on this pool.
set -euo pipefail
kind="${1:-thread}"
root="$(cd "$(dirname "$0")/.." && pwd)"
out="$root/build/san-$kind"
mkdir -p "$out"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
flags=(-std=c++17 -O1 -g -fPIC "-Xarch_host" "-fsanitize=$kind" -I"$root/include" -I"$root/dccl_amd/csrc" --offload-arch=gfx950)
objs=()
for f in comm algorithms grouped bootstrap dccl_api direct host_staged rccl_transport; do
  "$HIPCC" "${flags[@]}" -c "$root/dccl_amd/csrc/$f.cpp" -o "$out/$f.o"
  objs+=("$out/$f.o")
done
# the kernel translation units are reused from the normal build (their host side is launchers only)
lr=("$root/build/obj/local_reduce.hip.o" "$root/build/obj/phased_multi.hip.o" "$root/build/obj/phased_chain.hip.o"
    "$root/build/obj/unaligned_multi.hip.o")
for o in "${lr[@]}"; do [[ -f "$o" ]] || python "$root/dccl_amd/build.py" > /dev/null; done
"$HIPCC" "${flags[@]}" -c "$root/tools/dccl_cli.cpp" -o "$out/cli.o"
"$HIPCC" --offload-arch=gfx950 -Xarch_host "-fsanitize=$kind" "$out/cli.o" "${objs[@]}" "${lr[@]}" -o "$out/dccl_cli" -pthread -ldl
export TSAN_OPTIONS="halt_on_error=1 exitcode=66" ASAN_OPTIONS="halt_on_error=1 exitcode=66 detect_leaks=1" \
       UBSAN_OPTIONS="halt_on_error=1 exitcode=66 print_stacktrace=1"
run() { echo "+ dccl_cli $*"; "$out/dccl_cli" "$@" > "$out/last.log" 2>&1 || { cat "$out/last.log"; exit 1; }; }
run -a all_gather -t uint32 -c 4096 -n 4 -r 20 -g -1
run -a all_gather -t float64 -c 3003 -n 3 -r 5 -g -1
run -a broadcast -t int8 -c 65536 -n 8 -r 10 -g -1
run -a all_reduce -t float32 -c 1024 -n 1 -r 5 -g -1
run -a all_gather -t uint64 -c 8 -n 2 -r 50 -g -1
echo "sanitize_host($kind): clean"
