# round-3 GPU step ac: final build: C5 PMC passes, the default C2 bench under the kernel trace, N2 bench line
mkdir -p gpurun_out/r03ac
R=$GRAFT_REPO_ROOT
bash tools/pmc_workloads.sh r03ac c5 > gpurun_out/r03ac/pmc.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03ac/c2tr -o c2 -- python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r03ac/c2.json 2> $R/gpurun_out/r03ac/c2.err || exit 4
cd $R
timeout -k 10 300 python -u bench.py --workload n2 --steps 3 --warmup 1 > gpurun_out/r03ac/n2.json 2> gpurun_out/r03ac/n2.err || exit 5
