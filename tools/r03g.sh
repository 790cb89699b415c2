# round-3 GPU step g: MFMA GRID forward-backward probes (N1); V-scan tie list (C5)
mkdir -p gpurun_out/r03g
timeout -k 10 300 python -u -m pytest tests/test_gpu_large_k.py -q -k mfma --maxfail=5 --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03g/lk.log 2>&1
rc=$?; echo LK_EXIT $rc >> gpurun_out/r03g/lk.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 400 python -u -m pytest tests/test_gpu_vscan.py tests/test_gpu_configs.py tests/test_gpu_golden.py -q -k "vscan or c5 or tayal or golden" --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03g/vs.log 2>&1
rc=$?; echo VS_EXIT $rc >> gpurun_out/r03g/vs.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03g/c5.json 2>/dev/null || exit 4
for F in 0 131072; do
  for PARS in loglik,gamma_tk loglik; do
    timeout -k 10 200 python bench.py --workload n1 --steps 3 --warmup 1 --no-cpu-baseline --flags $F --pars $PARS > gpurun_out/r03g/n1_${F}_${PARS}.json 2>/dev/null || exit 4
  done
done
