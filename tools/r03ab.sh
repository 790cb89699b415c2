# round-3 GPU step ab: final build: whole GPU suite, smoke, every workload's bench line with its CPU baseline
mkdir -p gpurun_out/r03ab
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03ab/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> gpurun_out/r03ab/pytest.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ab/smoke.log 2>&1 || exit 4
bash tools/round_bench.sh r03ab > gpurun_out/r03ab/rb.log 2>&1 || exit 5
