# round-3 GPU step i: phased sweep (HHMM_FLAG_VFB) parity + C2 schedule A/B; C5 V-scan tie list A/B; lkm opt-in tests
mkdir -p gpurun_out/r03i
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_golden.py tests/test_gpu_large_k.py tests/test_gpu_devset.py -q -k "vfb or split or near_impossible or c2 or mfma or golden or devset" --maxfail=10 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03i/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> gpurun_out/r03i/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 300 python -u tools/ab_sched.py two vfb fused split > gpurun_out/r03i/ab_sched.json 2> gpurun_out/r03i/ab_sched.err || exit 4
timeout -k 10 400 python -u tools/ab_workload.py --workload c5 head=gsoc17-hhmm_amd/lib/libhhmm.so tieinl=gsoc17-hhmm_amd/lib/variants/libhhmm_tieinl.so --rounds 5 --steps 2 > gpurun_out/r03i/ab_c5.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --schedule vfb --no-cpu-baseline > gpurun_out/r03i/c2_vfb.json 2> gpurun_out/r03i/c2_vfb.err || exit 6
