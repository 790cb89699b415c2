#!/bin/bash
# C2 schedule timings, position check (via gpurun): ab_bench with the head library
# twice (head, head2 = a copy) beside the no-check build and round 4, then a kernel
# trace of head vs the no-check build in one process.
# Usage: tools/r05_ab4.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp
L=gsoc17-hhmm_amd/lib
V=$L/variants
timeout -k 10 300 python3 tools/ab_bench.py head=$L/libhhmm.so nochk=$V/libhhmm_nochk.so head2=$V/libhhmm_head2.so r04=$V/libhhmm_r04.so --rounds 7 > $O/ab_c2.log 2>&1 || { echo "ab c2 rc=$?"; tail -n 20 $O/ab_c2.log; exit 1; }
echo "ab c2 ok"; tail -n 5 $O/ab_c2.log | cut -c1-400
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o trace -- python3 tools/ab_bench.py head=$L/libhhmm.so nochk=$V/libhhmm_nochk.so --rounds 4 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -n 20 $O/trace.log; exit 1; }
echo "trace ok"
python3 tools/trace_by_variant.py $O/trace
