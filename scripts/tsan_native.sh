#!/bin/bash
# Host-side ThreadSanitizer build + run of the native PS server stress test (SURVEY §5.2 c).
# CPU only (the server has no device code).  Usage: scripts/tsan_native.sh [workers rounds keys]
set -e
cd "$(dirname "$0")/.."
mkdir -p build
if [ "${1:-}" = "async" ]; then  # async-PS control protocol (csrc/include/async_ctl.h)
  ${CXX:-/opt/rocm/lib/llvm/bin/clang++} -std=c++17 -O1 -g -fsanitize=thread -fno-omit-frame-pointer -pthread \
      -Icsrc/include csrc/runtime/tests/async_ctl_stress.cpp -o build/async_ctl_stress_tsan
  TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" ./build/async_ctl_stress_tsan "${2:-3}" "${3:-200}" "${4:-1}"
  exit $?
fi
${CXX:-/opt/rocm/lib/llvm/bin/clang++} -std=c++17 -O1 -g -fsanitize=thread -fno-omit-frame-pointer -pthread -Icsrc/runtime \
    csrc/runtime/ps_server.cpp csrc/runtime/tests/ps_stress.cpp -o build/ps_stress_tsan
TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" ./build/ps_stress_tsan "${1:-4}" "${2:-20}" "${3:-16}"
