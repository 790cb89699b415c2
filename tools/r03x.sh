# round-3 GPU step x: instruction-fetch counters of the C2 phased sweep (vfb_kernel is 110 KB of code)
mkdir -p gpurun_out/r03x
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03x
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1
grep -o 'SQC_[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_CYCLES[A-Z_]*\|SQ_INSTS_[A-Z_]*' $OUT/avail.txt | sort -u > $OUT/sq_names.txt
i=0
for CTRS in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
            "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-include-regex "vfb_kernel|fb_kernel|viterbi_kernel" --output-format csv -d $OUT/p$i -o p$i -- python $R/bench.py --no-cpu-baseline --no-check --no-path-gather --steps 1 --warmup 0 > $OUT/p$i.log 2>&1
  echo "pass $i rc=$?" >> $OUT/passes.txt
done
exit 0
