#!/bin/bash
# ASan + UBSan build and run of the host runtime (csrc/tests/host_sanitize.cpp).  CPU only.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-build/sanitize}
mkdir -p "$OUT"
SRC="csrc/core/store.cpp csrc/core/persist.cpp csrc/core/codec.cpp csrc/core/broker.cpp csrc/core/loadgen.cpp csrc/core/frontend.cpp"
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
    -Icsrc/kernels csrc/tests/host_sanitize.cpp $SRC -o "$OUT/host_sanitize" -lssl -lcrypto -lpthread
rm -rf /tmp/cmq-sanitize
ASAN_OPTIONS=halt_on_error=1:detect_leaks=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    "$OUT/host_sanitize" /tmp/cmq-sanitize
