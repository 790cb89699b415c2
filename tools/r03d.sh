# round-3 GPU step d: the whole GPU suite, then per-workload kernel traces + PMC (VALU / MFMA / HBM)
mkdir -p gpurun_out/r03d
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03d/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> gpurun_out/r03d/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
bash tools/pmc_workloads.sh r03d c3 c4 c5 n1 n2
echo PMC_EXIT $? >> gpurun_out/r03d/pytest.log
