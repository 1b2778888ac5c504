#!/bin/bash
# Runs the host-side CPU tests (CEL evaluator, schema compiler, text / binary ingest, snapshot
# files, the C ABI surface) against libgck built with AddressSanitizer + UBSan (make ASAN=1).
# CPU only: no GPU sanitizers are involved. Extra arguments go to pytest.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
RT=$(echo /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so)
make -C "$ROOT/gochugaru_amd/csrc" ASAN=1 -j8 >/dev/null
cd "$ROOT"
GCK_LIBRARY="$ROOT/gochugaru_amd/libgck_asan.so" \
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
LD_PRELOAD="$RT" \
  python -m pytest -q -p no:cacheprovider -m "not gpu" \
    tests/test_cel.py tests/test_abi.py tests/test_rel.py tests/test_snapfile.py "$@"
