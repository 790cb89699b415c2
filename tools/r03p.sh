# round-3 GPU step p: every workload's bench line with its CPU baseline on this build, N2 evidence line
mkdir -p gpurun_out/r03p
bash tools/round_bench.sh r03p > gpurun_out/r03p/rb.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --workload n2 --steps 3 --warmup 1 > gpurun_out/r03p/n2.json 2> gpurun_out/r03p/n2.err || exit 4
