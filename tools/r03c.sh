# round-3 GPU step c: large-K scan / FFBS / log-profile parity, dense-wave list A/B, N2 timing
mkdir -p gpurun_out/r03c
timeout -k 10 500 python -u -m pytest tests/test_gpu_lkscan.py tests/test_gpu_large_k.py -q --maxfail=15 --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03c/lk.log 2>&1
rc=$?; echo LK_EXIT $rc >> gpurun_out/r03c/lk.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -k "near_impossible" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03c/renorm.log 2>&1
rc=$?; echo RN_EXIT $rc >> gpurun_out/r03c/renorm.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 300 python -u tools/ab_bench.py old=gsoc17-hhmm_amd/lib/variants/libhhmm_old.so new=gsoc17-hhmm_amd/lib/libhhmm.so --rounds 9 > gpurun_out/r03c/ab.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --workload n2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03c/n2.json 2> gpurun_out/r03c/n2.err
echo N2_EXIT $? >> gpurun_out/r03c/n2.err
