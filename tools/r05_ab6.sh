#!/bin/bash
# Round-5 pass (via gpurun): C4 A/B of the FFBS contract's det_exp -- the
# table form read from an LDS copy (working tree) against the table-free
# degree-13 form (variant predet) -- in the state-parallel sweep (default
# dispatch) and in the lane sweep (HHMM_FLAG_VIT_LANES = 8, global table).
# Usage: tools/r05_ab6.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
L=gsoc17-hhmm_amd/lib
V=$L/variants
timeout -k 10 300 python3 tools/ab_workload.py --workload c4 head=$L/libhhmm.so predet=$V/libhhmm_predet.so \
    headL=$L/libhhmm.so#8 predetL=$V/libhhmm_predet.so#8 --rounds 5 --steps 3 > $O/ab_c4.log 2>&1 \
    || { echo "ab c4 rc=$?"; tail -20 $O/ab_c4.log; exit 1; }
echo "ab c4 ok"; tail -3 $O/ab_c4.log
