#!/bin/bash
# Host sanitizers on CPU, no GPU needed:
#  1. the oracle's ASan + UBSan build (make -C oracle sanitize), driven by its
#     own tests (oracle vs transcription, golden fixtures, FFBS contract);
#  2. libhhmm.so with hhmm_api.cpp's host code under ASan + UBSan
#     (-Xarch_host, the device code unchanged), driven by tests/test_abi.py and
#     the host-side shard-plan test.
# Usage: tools/sanitize.sh [LOGDIR]  (default profiles/sanitize); exits non-zero on any report.
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
LOG=${1:-$ROOT/profiles/sanitize}
mkdir -p "$LOG"
cd "$ROOT"
ASAN_RT=$(gcc -print-file-name=libasan.so)
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:verify_asan_link_order=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
make -s -C oracle sanitize || exit 2
HHMM_ORACLE_SAN=1 LD_PRELOAD=$ASAN_RT timeout -k 10 1500 python -m pytest -q -p no:cacheprovider \
    tests/test_oracle.py tests/test_golden.py tests/test_ffbs.py tests/test_detmath.py tests/test_crlog.py \
    tests/test_features.py tests/test_forecast.py tests/test_params.py -m "not gpu" > "$LOG/oracle.log" 2>&1
rc1=$?
echo "oracle tests under ASan+UBSan: exit $rc1" | tee -a "$LOG/oracle.log"

# libhhmm.so with the host side of the C ABI instrumented
SANLIB=${TMPDIR:-/tmp}/libhhmm_hostsan.so  # ~200 MB: outside the tree, it never travels to a GPU box
TMP=$(mktemp -d)
mkdir -p "$TMP/gsoc17-hhmm_amd"
cp -r include "$TMP/"
cp -r gsoc17-hhmm_amd/csrc "$TMP/gsoc17-hhmm_amd/"
CLANG_RT=$(/opt/rocm/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
make -s -j8 -C "$TMP/gsoc17-hhmm_amd/csrc" OBJDIR="$TMP/obj" OUT="$SANLIB" \
    EXTRA="-g -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined -shared-libsan" \
    > "$LOG/hostsan_build.log" 2>&1 || { echo "hostsan build failed"; exit 2; }
rm -rf "$TMP"
HHMM_LIB="$SANLIB" LD_PRELOAD=$CLANG_RT timeout -k 10 900 python -m pytest -q -p no:cacheprovider \
    tests/test_abi.py tests/test_shard_plan.py -m "not gpu" > "$LOG/hostsan_abi.log" 2>&1
rc2=$?
echo "libhhmm host code under ASan+UBSan (test_abi, shard plan): exit $rc2" | tee -a "$LOG/hostsan_abi.log"
[ $rc1 -eq 0 ] && [ $rc2 -eq 0 ]
