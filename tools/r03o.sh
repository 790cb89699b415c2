# round-3 GPU step o: whole GPU suite (large-K IOHMM, segments, device set, phased C2 default)
mkdir -p gpurun_out/r03o
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03o/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> gpurun_out/r03o/pytest.log
