mkdir -p gpurun_out/r03a
timeout -k 10 240 python -u -m pytest tests/test_gpu_lkscan.py -q --maxfail=10 --timeout 200 --timeout-method thread -p no:cacheprovider -x > gpurun_out/r03a/lkscan.log 2>&1; echo LKSCAN_EXIT $? >> gpurun_out/r03a/lkscan.log
grep -q "LKSCAN_EXIT 0" gpurun_out/r03a/lkscan.log || grep -q "failed" gpurun_out/r03a/lkscan.log || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_lkscan.py > gpurun_out/r03a/pytest.log 2>&1; echo PYTEST_EXIT $? >> gpurun_out/r03a/pytest.log
timeout -k 10 120 python -u -m pytest tests/test_gpu_configs.py -m gpu -q -s -k "c5" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03a/c5.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err
echo done
