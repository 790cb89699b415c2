# round-3 GPU step n: IOHMM at large K (state-parallel groups) against the oracle
mkdir -p gpurun_out/r03n
timeout -k 10 500 python -u -m pytest tests/test_gpu_iohmm_large_k.py -q --maxfail=15 --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03n/lkio.log 2>&1
rc=$?; echo LKIO_EXIT $rc >> gpurun_out/r03n/lkio.log
