# round-3 GPU step q: HEAD after the container re-creation: whole GPU suite, smoke, default bench
mkdir -p gpurun_out/r03q
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03q/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> gpurun_out/r03q/pytest.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03q/smoke.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py > gpurun_out/r03q/bench.json 2> gpurun_out/r03q/bench.err || exit 5
