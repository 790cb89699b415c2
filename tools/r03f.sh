# round-3 GPU step f: MFMA forward-backward for GRID batches at large K (parity, N1 bench)
mkdir -p gpurun_out/r03f
timeout -k 10 400 python -u -m pytest tests/test_gpu_large_k.py -q --maxfail=10 --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03f/lk.log 2>&1
rc=$?; echo LK_EXIT $rc >> gpurun_out/r03f/lk.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 300 python bench.py --workload n1 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03f/n1.json 2> gpurun_out/r03f/n1.err || exit 4
timeout -k 10 300 python bench.py --workload n1 --steps 5 --warmup 2 --no-cpu-baseline --flags 131072 > gpurun_out/r03f/n1_off.json 2> gpurun_out/r03f/n1_off.err || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03f/n1trace -o n1 -- python $GRAFT_REPO_ROOT/bench.py --workload n1 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>&1
echo TRACE_EXIT $? >> $GRAFT_REPO_ROOT/gpurun_out/r03f/lk.log
