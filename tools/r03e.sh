# round-3 GPU step e: large-K parity after the blocked back-pointer layout; N1 / N2 bench lines; C2 profile
mkdir -p gpurun_out/r03e
timeout -k 10 400 python -u -m pytest tests/test_gpu_large_k.py tests/test_gpu_lkscan.py -q --maxfail=10 --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03e/lk.log 2>&1
rc=$?; echo LK_EXIT $rc >> gpurun_out/r03e/lk.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --workload n1 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03e/n1.json 2> gpurun_out/r03e/n1.err || exit 4
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03e/smoke.log 2>&1 || exit 5
bash tools/profile_box.sh r03e > gpurun_out/r03e/prof.log 2>&1
echo PROF_EXIT $? >> gpurun_out/r03e/prof.log
