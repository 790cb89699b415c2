# round-3 GPU step aa: C5 kernel trace (timeline of the two streams) on this build
mkdir -p gpurun_out/r03aa
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03aa
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o c5 -- python $R/bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err || exit 3
