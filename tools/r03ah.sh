# round-3 GPU step ah: HEAD's build (bound tied to the cadence): whole GPU suite and smoke
mkdir -p gpurun_out/r03ah
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03ah/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> gpurun_out/r03ah/pytest.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ah/smoke.log 2>&1 || exit 4
