#!/bin/bash
# Round-5 A/B pass (via gpurun): interleaved variant timings in one process per
# workload (tools/ab_workload.py), then the IOHMM log-space worst case.  Every
# step under its own time limit, chained: the first failure ends the call.
# Usage: tools/r05_ab.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
L=gsoc17-hhmm_amd/lib
V=$L/variants
ab() {
  w=$1; shift
  timeout -k 10 240 python3 tools/ab_workload.py --workload $w "$@" > $O/ab_$w.log 2>&1 || { echo "ab $w rc=$?"; tail -20 $O/ab_$w.log; exit 1; }
  echo "ab $w ok"; tail -4 $O/ab_$w.log
}
ab n2 head=$L/libhhmm.so mfma16=$V/libhhmm_mfma16.so --rounds 5 --steps 3 &&
ab c3 head=$L/libhhmm.so preziv=$V/libhhmm_preziv.so --rounds 5 --steps 3 &&
ab c4 head=$L/libhhmm.so predet=$V/libhhmm_predet.so --rounds 5 --steps 3 &&
ab c1 head=$L/libhhmm.so bound4=$V/libhhmm_bound4.so --rounds 7 --steps 20 &&
timeout -k 10 240 python3 tools/ab_bench.py head=$L/libhhmm.so r04=$V/libhhmm_r04.so --rounds 5 > $O/ab_c2.log 2>&1 || { echo "ab c2 rc=$?"; tail -20 $O/ab_c2.log; exit 1; }
echo "ab c2 ok"; tail -4 $O/ab_c2.log &&
timeout -k 10 300 python3 tools/iolog_worst.py > $O/iolog_worst.json 2> $O/iolog_worst.err || { echo "iolog rc=$?"; tail -20 $O/iolog_worst.err; exit 2; }
echo "iolog ok"; cat $O/iolog_worst.err
