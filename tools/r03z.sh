# round-3 GPU step z: lane-parallel approximate V-scan (vs_scan0_block): V-scan parity, C5 A/B against the serial walk, chunk stats
mkdir -p gpurun_out/r03z
L=gsoc17-hhmm_amd/lib/libhhmm.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_vscan.py tests/test_gpu_configs.py -k "vscan or c5 or tayal" -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03z/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> gpurun_out/r03z/pytest.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -u tools/ab_workload.py --workload c5 --rounds 7 --steps 2 par=$L serial=$L@HHMM_PROBE_VS_SCAN0_SERIAL=1 > gpurun_out/r03z/c5.log 2>&1 || exit 4
HHMM_PROBE_VS_STATS=1 timeout -k 10 200 python -u bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r03z/stats_par.json 2> gpurun_out/r03z/stats_par.err || exit 5
HHMM_PROBE_VS_STATS=1 HHMM_PROBE_VS_SCAN0_SERIAL=1 timeout -k 10 200 python -u bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r03z/stats_ser.json 2> gpurun_out/r03z/stats_ser.err || exit 6
