#!/bin/bash
# PMC passes (one run each) over one bench.py workload, restricted to kernels
# matching a regex.  Usage: tools/pmc_workload.sh TAG REGEX [bench args...]
TAG=$1; RX=$2; shift 2
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
            "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VALU_TRANS_F64"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $CTRS --kernel-include-regex "$RX" --output-format csv -d $OUT/p$i -o p$i -- python $R/bench.py --no-cpu-baseline --no-check --steps 1 --warmup 0 "$@" > $OUT/p$i.log 2>&1
  echo "pass $i rc=$?" >> $OUT/passes.txt
done
