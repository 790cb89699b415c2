#!/bin/bash
# Runs on the GPU box (via gpurun): kernel trace of the exact default bench
# command (same steps / warmup as the judged line) + separate PMC passes of a
# 1-step run, restricted to libhhmm's kernels.
# Usage: tools/profile_box.sh TAG [bench args for the PMC passes...]
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --no-cpu-baseline $*"
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $OUT/trace.log 2>&1 || exit 1
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
            "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64" \
            "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $CTRS --kernel-include-regex "hhmm" --output-format csv -d $OUT/pmc$i -o pmc$i -- python $BENCH > $OUT/pmc$i.log 2>&1
  echo "pass $i rc=$?" >> $OUT/passes.txt
done
exit 0
