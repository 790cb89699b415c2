# round-3 GPU step b: large-K scan parity, renormalisation-gate A/B, N2 timing
mkdir -p gpurun_out/r03b
timeout -k 10 400 python -u -m pytest tests/test_gpu_lkscan.py tests/test_gpu_large_k.py -q --maxfail=10 --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03b/lkscan.log 2>&1
rc=$?; echo LKSCAN_EXIT $rc >> gpurun_out/r03b/lkscan.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 300 python -u tools/ab_bench.py old=gsoc17-hhmm_amd/lib/variants/libhhmm_old.so cur=gsoc17-hhmm_amd/lib/variants/libhhmm_cur.so fix=gsoc17-hhmm_amd/lib/libhhmm.so --rounds 7 > gpurun_out/r03b/ab.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03b/n2trace -o n2 -- python $GRAFT_REPO_ROOT/bench.py --workload n2 --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r03b/n2.json 2> $GRAFT_REPO_ROOT/gpurun_out/r03b/n2.err
echo N2_EXIT $? >> $GRAFT_REPO_ROOT/gpurun_out/r03b/n2.err
