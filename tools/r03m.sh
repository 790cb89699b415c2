# round-3 GPU step m: segment windows (one series split along T over ranks), device set, then the whole suite
mkdir -p gpurun_out/r03m
timeout -k 10 400 python -u -m pytest tests/test_gpu_segment.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03m/seg.log 2>&1
rc=$?; echo SEG_EXIT $rc >> gpurun_out/r03m/seg.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03m/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> gpurun_out/r03m/pytest.log
