#!/bin/bash
# C2 regression hunt (via gpurun): the device entry's data checks A/B'd against
# the round-4 library in one process (tools/ab_bench.py), a kernel trace of the
# head library's schedules, then C5 and C1 head vs round 4.
# Usage: tools/r05_ab2.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp
L=gsoc17-hhmm_amd/lib
V=$L/variants
timeout -k 10 300 python3 tools/ab_bench.py head=$L/libhhmm.so nochk=$V/libhhmm_nochk.so noxc=$V/libhhmm_noxc.so r04=$V/libhhmm_r04.so --rounds 7 > $O/ab_c2.log 2>&1 || { echo "ab c2 rc=$?"; tail -20 $O/ab_c2.log; exit 1; }
echo "ab c2 ok"; tail -n 5 $O/ab_c2.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 tools/ab_bench.py head=$L/libhhmm.so --rounds 2 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -20 $O/trace.log; exit 1; }
echo "trace ok"
ab() {
  w=$1; shift
  timeout -k 10 240 python3 tools/ab_workload.py --workload $w "$@" > $O/ab_$w.log 2>&1 || { echo "ab $w rc=$?"; tail -20 $O/ab_$w.log; exit 1; }
  echo "ab $w ok"; tail -n 4 $O/ab_$w.log
}
ab c5 head=$L/libhhmm.so r04=$V/libhhmm_r04.so --rounds 5 --steps 3 &&
ab c1 head=$L/libhhmm.so r04=$V/libhhmm_r04.so --rounds 7 --steps 20
