#!/bin/bash
# Round-5 pass (via gpurun): the det_exp table read from LDS in every FFBS
# sweep (working tree) against the table-free degree-13 form (variant predet):
# C4 in the state-parallel and the lane sweep, and the Gaussian HMM's FFBS in
# fb_kernel (C1's shape with z_ffbs requested); N2 with the chunk products
# renormalised every 4th step; N1 / N2 with lk_fb_kernel renormalising every
# 8th step (variant lkr4: every 4th).  Then the GPU suite + smoke.
# Usage: tools/r05_ab7.sh TAG
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
echo "ab c4 ok"; tail -1 $O/ab_c4.log
timeout -k 10 200 python3 tools/ab_workload.py --workload c1 --pars loglik,gamma_tk,z_ffbs head=$L/libhhmm.so \
    predet=$V/libhhmm_predet.so --rounds 7 --steps 20 > $O/ab_c1_ffbs.log 2>&1 \
    || { echo "ab c1 rc=$?"; tail -20 $O/ab_c1_ffbs.log; exit 2; }
echo "ab c1 ffbs ok"; tail -1 $O/ab_c1_ffbs.log
timeout -k 10 300 python3 tools/ab_workload.py --workload n2 head=$L/libhhmm.so predet=$V/libhhmm_predet.so \
    lkr4=$V/libhhmm_lkr4.so --rounds 4 --steps 2 > $O/ab_n2.log 2>&1 || { echo "ab n2 rc=$?"; tail -20 $O/ab_n2.log; exit 5; }
echo "ab n2 ok"; tail -1 $O/ab_n2.log
timeout -k 10 300 python3 tools/ab_workload.py --workload n1 head=$L/libhhmm.so lkr4=$V/libhhmm_lkr4.so \
    --rounds 5 --steps 3 > $O/ab_n1.log 2>&1 || { echo "ab n1 rc=$?"; tail -20 $O/ab_n1.log; exit 6; }
echo "ab n1 ok"; tail -1 $O/ab_n1.log
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "suite rc=$?"; tail -40 $O/pytest.log; exit 3; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 4; }
echo "smoke ok"
