# round-3 GPU step k: waits restructured (copy-at-top prefetch, drained loop entries, predicate-free full blocks)
mkdir -p gpurun_out/r03k
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03k/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> gpurun_out/r03k/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 400 python -u tools/ab_sched.py --lib new=gsoc17-hhmm_amd/lib/libhhmm.so --lib base=gsoc17-hhmm_amd/lib/variants/libhhmm_base.so new:vfb base:vfb new:two base:two > gpurun_out/r03k/ab_sched.json 2> gpurun_out/r03k/ab_sched.err || exit 4
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03k/c2.json 2> gpurun_out/r03k/c2.err || exit 5
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03k/c5.json 2> gpurun_out/r03k/c5.err || exit 6
