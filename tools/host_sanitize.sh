#!/bin/bash
# AddressSanitizer + UBSan build of libgnnd's HOST code (graph builder, table validation):
# -fsanitize applies to the host compilation only (-Xarch_host), the device code is
# unchanged.  Runs tools/host_check.cpp on random graphs; no GPU needed.
# usage: tools/host_sanitize.sh [OUTDIR] [GRAPHS]
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${1:-/tmp/gnnd_hostsan}"; N="${2:-300}"
mkdir -p "$OUT"
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all"
/opt/rocm/bin/hipcc -O1 -g -std=c++17 --offload-arch=gfx950 $SAN \
  "$ROOT/gnn-decode_amd/csrc/gnnd_graph.hip" "$ROOT/tools/host_check.cpp" -o "$OUT/host_check"
ASAN_OPTIONS=detect_leaks=1 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/host_check" "$N"
