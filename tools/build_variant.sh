#!/bin/bash
# Builds libhhmm.so from a git revision (or the working tree with REV=WT) into
# gsoc17-hhmm_amd/lib/variants/libhhmm_NAME.so, for tools/ab_bench.py.
# Usage: tools/build_variant.sh NAME REV [make variables, e.g. EXTRA="-DHHMM_PROBES" for the HHMM_PROBE_* knobs]
set -e
NAME=$1; REV=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
if [ "$REV" = "WT" ]; then
  # sources only: copying lib/obj would give stale objects fresh mtimes
  mkdir -p "$TMP/gsoc17-hhmm_amd"
  cp -r "$ROOT/include" "$TMP/"
  cp -r "$ROOT/gsoc17-hhmm_amd/csrc" "$TMP/gsoc17-hhmm_amd/"
else
  (cd "$ROOT" && git archive "$REV" include gsoc17-hhmm_amd/csrc) | tar -x -C "$TMP"
fi
mkdir -p "$ROOT/gsoc17-hhmm_amd/lib/variants"
make -s -j8 -C "$TMP/gsoc17-hhmm_amd/csrc" OUT="$ROOT/gsoc17-hhmm_amd/lib/variants/libhhmm_$NAME.so" "$@"
rm -rf "$TMP"
echo "built libhhmm_$NAME.so from $REV"
