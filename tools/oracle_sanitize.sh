#!/bin/bash
# Runs the oracle's CPU tests against the ASan/UBSan build of oracle/oracle.cpp.
# Host code only (no GPU): libasan is preloaded into the test interpreter because python itself is
# not instrumented; leak checking is off (the interpreter's own allocations are not ours).
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -C oracle asan
export ORACLE_LIB="$PWD/oracle/build/liboracle_asan.so"
export LD_PRELOAD="$(g++ -print-file-name=libasan.so):$(g++ -print-file-name=libubsan.so)"
export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
exec python -m pytest -q -p no:cacheprovider tests/test_cpu_oracle_golden.py tests/test_cpu_distributed.py "$@"
