# round-3 GPU step ag: C2 phased sweep renormalising every 8 steps (bound 2^-19) against every 4: A/B, then parity with the 8-step build
mkdir -p gpurun_out/r03ag
N=gsoc17-hhmm_amd/lib/variants/libhhmm_rn8.so; B=gsoc17-hhmm_amd/lib/libhhmm.so
timeout -k 10 400 python -u tools/ab_sched.py --lib base=$B --lib rn8=$N --rounds 9 --steps 3 base:vfb rn8:vfb > gpurun_out/r03ag/ab.json 2> gpurun_out/r03ag/ab.err || exit 3
HHMM_LIB=$N timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_golden.py -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03ag/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> gpurun_out/r03ag/pytest.log
exit $rc
