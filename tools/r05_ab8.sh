#!/bin/bash
# Round-5 pass (via gpurun): the large-K gamma test that the 8-step cadence
# failed (kGammaDirect = 2^-240 now), the GPU suite + smoke, then C5 and C2
# A/B against the round's first build (variant predet): the direct-gamma
# threshold is in their kernels too.  N2: lks_prod_kernel's full-block
# specialisation and tiles per wave (t2nf / t1nf / t1 variants).
# Usage: tools/r05_ab8.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
L=gsoc17-hhmm_amd/lib
V=$L/variants
timeout -k 10 200 python -u -m pytest tests/test_gpu_large_k.py -m gpu -q -x --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $O/large_k.log 2>&1 || { echo "large_k rc=$?"; tail -30 $O/large_k.log; exit 1; }
tail -1 $O/large_k.log
timeout -k 10 300 python3 tools/ab_workload.py --workload n2 head=$L/libhhmm.so t2nf=$V/libhhmm_t2nf.so \
    t1nf=$V/libhhmm_t1nf.so t1=$V/libhhmm_t1.so --rounds 3 --steps 2 > $O/ab_n2.log 2>&1 \
    || { echo "ab n2 rc=$?"; tail -20 $O/ab_n2.log; exit 6; }
echo "ab n2 ok"; tail -1 $O/ab_n2.log
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "suite rc=$?"; tail -40 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 3; }
echo "smoke ok"
timeout -k 10 300 python3 tools/ab_workload.py --workload c5 head=$L/libhhmm.so predet=$V/libhhmm_predet.so \
    --rounds 5 --steps 3 > $O/ab_c5.log 2>&1 || { echo "ab c5 rc=$?"; tail -20 $O/ab_c5.log; exit 4; }
echo "ab c5 ok"; tail -1 $O/ab_c5.log
timeout -k 10 300 python3 tools/ab_bench.py head=$L/libhhmm.so predet=$V/libhhmm_predet.so --rounds 5 > $O/ab_c2.log 2>&1 \
    || { echo "ab c2 rc=$?"; tail -20 $O/ab_c2.log; exit 5; }
echo "ab c2 ok"; tail -1 $O/ab_c2.log
