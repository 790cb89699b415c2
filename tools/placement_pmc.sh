#!/bin/bash
# The C2 placement probe, plain then under three rocprofv3 --pmc passes (each
# its own process: the placements differ per process, the per-set counters are
# read within each pass).  Usage: tools/placement_pmc.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tools/placement_probe.py --sets 5 --fb --rounds 2 --steps 1"
i=0
for C in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCC_WRITE_REQ_LATENCY_sum" \
         "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" \
         "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/pmc$i -o pmc -- $P > $O/probe_pmc$i.log 2>&1 \
      || { echo "pmc pass $i rc=$?"; tail -5 $O/probe_pmc$i.log; exit 1; }
  python3 $R/tools/placement_pmc.py $O/pmc$i 5 $O/placement_pmc$i.json > /dev/null || exit 2
  rm -rf $O/pmc$i
  grep spread_pct $O/probe_pmc$i.log
done
echo done
