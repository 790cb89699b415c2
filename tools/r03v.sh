# round-3 GPU step v: side-stream priority + 1M-lane small-batch T-chunks: scan / V-scan / segment / C5 tests, C5 and N2 bench lines
mkdir -p gpurun_out/r03v
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_scan.py tests/test_gpu_vscan.py tests/test_gpu_segment.py tests/test_gpu_lkscan.py -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03v/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> gpurun_out/r03v/pytest.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 2 > gpurun_out/r03v/c5.json 2> gpurun_out/r03v/c5.err || exit 4
timeout -k 10 300 python -u bench.py --workload n2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03v/n2.json 2> gpurun_out/r03v/n2.err || exit 5
