#!/bin/bash
# CPU test suite under AddressSanitizer + UBSan: the oracle
# (oracle/liboracle_asan.so) and the C ABI's host code (libsechs_asan.so,
# -Xarch_host sanitizers; device code unchanged) -- run in the build
# container:  bash tools/asan_cpu.sh
set -eo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
make -s -C $R/oracle asan
make -s -j8 -C $R/rl-6-nimmt_amd libsechs_asan.so
ASAN_RT=$(gcc -print-file-name=libasan.so)
UBSAN_RT=$(gcc -print-file-name=libubsan.so)
HIP_ASAN=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so 2>/dev/null || true)
cd $R
# the oracle is gcc-built (libasan), the ABI library clang-built (its own runtime): one run per runtime
LD_PRELOAD="$ASAN_RT $UBSAN_RT" ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  SECHS_ORACLE_LIB=$R/oracle/liboracle_asan.so python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider \
  tests/test_oracle_golden.py tests/test_league_cpu.py tests/test_evolve_cpu.py tests/test_distributed_cpu.py
if [ -n "$HIP_ASAN" ] && [ -f "$HIP_ASAN" ]; then
  LD_PRELOAD="$HIP_ASAN" ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 \
    SECHS_LIB=$R/rl-6-nimmt_amd/libsechs_asan.so python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider \
    tests/test_abi_cpu.py tests/test_league_cpu.py tests/test_evolve_cpu.py
fi
echo "asan: clean"
