#!/usr/bin/env bash
# SURVEY.md §5 "Race detection / sanitizers", host side (no GPU sanitizers exist on this pool):
#   1. the C++ oracle built with ASan + UBSan (oracle/Makefile.asan -> liboracle_asan.so);
#   2. libfvo's C-ABI argument / config validation (csrc/capi.cpp) built host-only with ASan +
#      UBSan against a stub device layer (tests/sanitize/) and run;
#   3. the CPU test suite (pytest -m "not gpu") with the instrumented oracle loaded
#      (FVO_ORACLE_LIB) and the ASan runtime preloaded into the Python process.
# Run in the CPU container:  bash tools/sanitize.sh  -> exit 0 when every leg is clean.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/build/sanitize"
mkdir -p "$OUT"
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1"
export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:strict_init_order=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"

echo "== 1. oracle (ASan + UBSan)"
make -s -C "$ROOT/oracle" -f Makefile.asan -B

echo "== 2. C ABI validation, host-only (ASan + UBSan)"
g++ -std=c++17 $SAN -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I"$ROOT/include" \
    "$ROOT/forest-slam_amd/csrc/capi.cpp" "$ROOT/tests/sanitize/host_stubs.cpp" "$ROOT/tests/sanitize/capi_check.cpp" \
    -o "$OUT/capi_check"
"$OUT/capi_check"

echo "== 3. CPU test suite with the instrumented oracle"
ASAN_RT="$(g++ -print-file-name=libasan.so)"
cd "$ROOT"
LD_PRELOAD="$ASAN_RT${LD_PRELOAD:+:$LD_PRELOAD}" FVO_ORACLE_LIB="$ROOT/oracle/liboracle_asan.so" \
    python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
