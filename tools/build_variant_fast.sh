#!/bin/bash
# A build-knob variant of the working tree's libhhmm.so that recompiles only
# the named translation units (the rest reuse lib/obj, which must be current):
# gsoc17-hhmm_amd/lib/variants/libhhmm_NAME.so, for tools/ab_workload.py.
# Usage: tools/build_variant_fast.sh NAME "EXTRA flags" unit.hip [unit.hip ...]
set -e
NAME=$1; FLAGS=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
cp -a "$ROOT/gsoc17-hhmm_amd/lib/obj/." "$TMP/"
for u in "$@"; do rm -f "$TMP/$u.o"; done
mkdir -p "$ROOT/gsoc17-hhmm_amd/lib/variants"
make -s -j8 -C "$ROOT/gsoc17-hhmm_amd/csrc" OBJDIR="$TMP" OUT="$ROOT/gsoc17-hhmm_amd/lib/variants/libhhmm_$NAME.so" EXTRA="$FLAGS"
rm -rf "$TMP"
echo "built libhhmm_$NAME.so ($FLAGS; rebuilt $*)"
