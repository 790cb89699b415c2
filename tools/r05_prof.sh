#!/bin/bash
# Round-5 profiling pass (via gpurun): N2 tile-count A/B, then rocprofv3 kernel
# traces of short bench runs of the evidence workloads (per-kernel times of the
# current build).  Every step under its own time limit; the first failure ends it.
# Usage: tools/r05_prof.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
L=gsoc17-hhmm_amd/lib
V=$L/variants
timeout -k 10 300 python3 tools/ab_workload.py --workload n2 t2=$L/libhhmm.so t3=$V/libhhmm_tiles3.so t4=$V/libhhmm_tiles4.so --rounds 4 --steps 2 > $O/ab_n2_tiles.log 2>&1 || { echo "ab n2 rc=$?"; tail -20 $O/ab_n2_tiles.log; exit 1; }
echo "ab n2 tiles ok"; tail -1 $O/ab_n2_tiles.log
cd /tmp && export TMPDIR=/tmp
for w in n2 c5 c4 c3 n1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$w -o trace -- \
      python3 $R/bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err \
      || { echo "trace $w rc=$?"; tail -20 $O/bench_$w.err; exit 2; }
  echo "trace $w ok"
done
exit 0
