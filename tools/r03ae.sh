# round-3 GPU step ae: T-scan chunk products renormalised every 4 steps where the parameters bound the shrink: parity and C5 / C1 A/B
mkdir -p gpurun_out/r03ae
L=gsoc17-hhmm_amd/lib/variants/libhhmm_scanrn.so; B=gsoc17-hhmm_amd/lib/libhhmm.so
HHMM_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_scan.py tests/test_gpu_vscan.py tests/test_gpu_segment.py tests/test_gpu_parity.py tests/test_gpu_golden.py -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03ae/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> gpurun_out/r03ae/pytest.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -u tools/ab_workload.py --workload c5 --rounds 7 --steps 2 new=$L base=$B > gpurun_out/r03ae/c5.log 2>&1 || exit 4
