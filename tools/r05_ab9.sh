#!/bin/bash
# Round-5 pass (via gpurun): lk_fb_kernel with split columns (a pair per wave,
# each half of the wave half of the K-vectors' index range; HHMM_LK_SPLIT)
# and lk_viterbi_kernel likewise (HHMM_LK_VSPLIT) -- the large-K / scan /
# segment GPU tests, then N1 and N2 against the variants novs (the Viterbi
# unsplit) and nosplit (neither kernel split).
# Usage: tools/r05_ab9.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
L=gsoc17-hhmm_amd/lib
V=$L/variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_large_k.py tests/test_gpu_lkscan.py tests/test_gpu_segment.py \
    tests/test_gpu_configs.py -k "large or lk or K or n1 or n2 or segment" -m gpu -q -x --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $O/large_k.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/large_k.log; exit 1; }
tail -1 $O/large_k.log
timeout -k 10 300 python3 tools/ab_workload.py --workload n1 head=$L/libhhmm.so novs=$V/libhhmm_novs.so nosplit=$V/libhhmm_nosplit.so \
    --rounds 5 --steps 3 > $O/ab_n1.log 2>&1 || { echo "ab n1 rc=$?"; tail -20 $O/ab_n1.log; exit 2; }
echo "ab n1 ok"; tail -1 $O/ab_n1.log
timeout -k 10 300 python3 tools/ab_workload.py --workload n2 head=$L/libhhmm.so nosplit=$V/libhhmm_nosplit.so \
    --rounds 4 --steps 2 > $O/ab_n2.log 2>&1 || { echo "ab n2 rc=$?"; tail -20 $O/ab_n2.log; exit 3; }
echo "ab n2 ok"; tail -1 $O/ab_n2.log
