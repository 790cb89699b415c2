#!/bin/bash
# Final build, pass A (via gpurun): PMC evidence keyed to the build --
# the judged C2 command under rocprofv3 --kernel-trace --stats (one process:
# its JSON line and the trace it produced), FETCH_SIZE and WRITE_SIZE passes
# of a 1-step C2 run (each its own rocprofv3 run), then the per-workload
# trace + PMC passes of tools/pmc_workloads.sh.  Stops at the first failure.
# Usage: tools/final_pass_a.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/trace.log 2> $OUT/trace.err \
    || { echo "traced bench rc=$?"; tail -20 $OUT/trace.err; exit 1; }
echo "traced bench ok"
BENCH="$R/bench.py --no-cpu-baseline --no-check --no-path-gather --steps 1 --warmup 1"
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $CTRS --kernel-include-regex "hhmm" --output-format csv -d $OUT/pmc$i -o pmc$i \
      -- python3 $BENCH > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i rc=$?"; tail -20 $OUT/pmc$i.log; exit 2; }
  echo "pmc pass $i ok"
done
bash $R/tools/pmc_workloads.sh $TAG c3 c4 c5 n1 n2 || { echo "workload pmc failed"; cat $R/gpurun_out/pmcw_$TAG/passes.txt; exit 3; }
echo "workload pmc ok"
