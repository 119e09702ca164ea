#!/bin/bash
# Build the native CPU runtime + its self-test with AddressSanitizer and UBSan and run it
# (SURVEY.md §5.2).  Host code only: GPU ASan / xnack+ builds are not available on this pool.
set -euo pipefail
REPO="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${1:-/tmp/dmlc_sanitize}"
mkdir -p "$OUT"
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
    -pthread -I"$REPO/csrc/runtime" \
    "$REPO"/csrc/runtime/crc_coding.cpp "$REPO"/csrc/runtime/tensor_bundle.cpp "$REPO"/csrc/runtime/records_cifar.cpp \
    "$REPO"/csrc/runtime/tests/rt_selftest.cpp -o "$OUT/rt_selftest"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/rt_selftest" "$OUT"
