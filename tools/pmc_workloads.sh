#!/bin/bash
# Runs on the GPU box (via gpurun): for each bench.py workload named on the
# command line, one kernel-trace pass and two PMC passes (HBM bytes, VALU /
# MFMA instruction counts) of a 1-step run, each in its own rocprofv3 run
# under its own time limit.  Output: gpurun_out/pmcw_TAG/<workload>/...
# Usage: tools/pmc_workloads.sh TAG c3 c4 c5 n1 n2
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmcw_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for W in "$@"; do
  D=$OUT/$W
  mkdir -p $D
  ARGS="$R/bench.py --workload $W --no-cpu-baseline --no-check --no-sequential --no-path-gather --steps 1 --warmup 1"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o trace -- python $ARGS > $D/trace.log 2>&1
  rc=$?; echo "$W trace rc=$rc" >> $OUT/passes.txt; [ $rc -eq 0 ] || exit 1
  i=0
  for CTRS in "FETCH_SIZE SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES GRBM_GUI_ACTIVE" \
              "WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_SALU SQ_INSTS_LDS"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $CTRS --kernel-include-regex "hhmm" --output-format csv -d $D/pmc$i -o pmc$i -- python $ARGS > $D/pmc$i.log 2>&1
    rc=$?; echo "$W pass $i rc=$rc" >> $OUT/passes.txt; [ $rc -eq 0 ] || exit 1
  done
done
exit 0
