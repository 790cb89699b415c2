# round-3 GPU step h (re-entry): whole GPU suite on HEAD, smoke, C2 / N1 / C5 / N2 bench lines
mkdir -p gpurun_out/r03h
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03h/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> gpurun_out/r03h/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03h/smoke.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03h/c2.json 2> gpurun_out/r03h/c2.err || exit 4
timeout -k 10 300 python bench.py --workload n1 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03h/n1.json 2> gpurun_out/r03h/n1.err || exit 4
timeout -k 10 300 python bench.py --workload n1 --steps 5 --warmup 2 --no-cpu-baseline --flags 131072 > gpurun_out/r03h/n1_off.json 2> gpurun_out/r03h/n1_off.err || exit 4
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03h/c5.json 2> gpurun_out/r03h/c5.err || exit 4
timeout -k 10 300 python bench.py --workload n2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03h/n2.json 2> gpurun_out/r03h/n2.err || exit 4
