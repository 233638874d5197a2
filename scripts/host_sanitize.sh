#!/bin/bash
# Host runtime under sanitizers (csrc/tests/host_sanitize.cpp), CPU only:
#   1. AddressSanitizer + UndefinedBehaviorSanitizer (g++)
#   2. ThreadSanitizer (clang++ from the ROCm LLVM: gcc 11's libtsan does not intercept
#      pthread_cond_clockwait, which std::condition_variable::wait_for uses, and then
#      reports mutexes held across waits as double locks / races)
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-build/sanitize}
mkdir -p "$OUT"
SRC="csrc/core/store.cpp csrc/core/bodylog.cpp csrc/core/persist.cpp csrc/core/codec.cpp csrc/core/broker.cpp csrc/core/loadgen.cpp csrc/core/frontend.cpp"
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
    -Icsrc/kernels csrc/tests/host_sanitize.cpp $SRC -o "$OUT/host_sanitize" -lssl -lcrypto -lpthread
rm -rf /tmp/cmq-sanitize
echo "== ASan + UBSan"
ASAN_OPTIONS=halt_on_error=1:detect_leaks=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    "$OUT/host_sanitize" /tmp/cmq-sanitize
/opt/rocm/lib/llvm/bin/clang++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=thread \
    -Icsrc/kernels csrc/tests/host_sanitize.cpp $SRC -o "$OUT/host_tsan" -lssl -lcrypto -lpthread
rm -rf /tmp/cmq-tsan
echo "== TSan"
TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 "$OUT/host_tsan" /tmp/cmq-tsan
