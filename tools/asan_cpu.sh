#!/bin/bash
# The CPU test suite against AddressSanitizer + UBSan builds of the host C++ / C-ABI
# (sparkglm_amd/lib_asan) and of the oracle (oracle/build/libsglm_oracle_asan.so).
# CPU only: GPU sanitizers are not available on this pool.
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$ROOT/sparkglm_amd/csrc" asan -j8 >/dev/null || exit 1
make -s -C "$ROOT/oracle" asan >/dev/null || exit 1
RT=$(ls /opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export SGLM_LIB="$ROOT/sparkglm_amd/lib_asan/libsglm_hip.so"
export SGLM_ORACLE_LIB="$ROOT/oracle/build/libsglm_oracle_asan.so"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
cd "$ROOT" && LD_PRELOAD="$RT" python -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@"
