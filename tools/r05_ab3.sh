#!/bin/bash
# Inline data checks (via gpurun): the invalid-data GPU tests, then C2's schedules
# A/B'd against the library without checks and the round-4 library (one process).
# Usage: tools/r05_ab3.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
L=gsoc17-hhmm_amd/lib
V=$L/variants
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_invalid_data.py > $O/invalid_data.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/invalid_data.log; exit 1; }
echo "tests ok"; tail -n 2 $O/invalid_data.log
timeout -k 10 300 python3 tools/ab_bench.py head=$L/libhhmm.so nochk=$V/libhhmm_nochk.so r04=$V/libhhmm_r04.so --rounds 7 > $O/ab_c2.log 2>&1 || { echo "ab c2 rc=$?"; tail -n 20 $O/ab_c2.log; exit 1; }
echo "ab c2 ok"; tail -n 4 $O/ab_c2.log
