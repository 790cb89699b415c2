#!/bin/bash
# Placement controls (via gpurun): C2 variants on shared buffers (tools/ab_bench.py),
# then C4 with the det_exp table build between two copies of the head library.
# Usage: tools/r05_ab5.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
L=gsoc17-hhmm_amd/lib
V=$L/variants
timeout -k 10 300 python3 tools/ab_bench.py head=$L/libhhmm.so nochk=$V/libhhmm_nochk.so head2=$V/libhhmm_head2.so r04=$V/libhhmm_r04.so --rounds 7 > $O/ab_c2.log 2>&1 || { echo "ab c2 rc=$?"; tail -n 20 $O/ab_c2.log; exit 1; }
echo "ab c2 ok"; tail -n 5 $O/ab_c2.log | cut -c1-420
timeout -k 10 300 python3 tools/ab_workload.py --workload c4 head=$L/libhhmm.so dettab=$V/libhhmm_dettab.so head2=$V/libhhmm_head2.so --rounds 5 --steps 3 > $O/ab_c4.log 2>&1 || { echo "ab c4 rc=$?"; tail -n 20 $O/ab_c4.log; exit 1; }
echo "ab c4 ok"; tail -n 1 $O/ab_c4.log
