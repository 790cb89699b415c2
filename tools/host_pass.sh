#!/bin/bash
# c2-host bench plain, then under rocprofv3 kernel + memory-copy trace, then the overlap summary.
# Usage: tools/host_pass.sh TAG [extra bench args]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u bench.py --workload c2-host --steps 3 --warmup 1 "$@" > $O/bench_host.json 2> $O/bench_host.err \
    || { echo "host bench rc=$?"; tail -20 $O/bench_host.err; exit 5; }
echo "host bench ok"; cat $O/bench_host.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace -o trace -- \
    python3 $R/bench.py --workload c2-host --steps 3 --warmup 1 "$@" > $O/bench_host_traced.json 2> $O/bench_host_traced.err \
    || { echo "traced host bench rc=$?"; tail -20 $O/bench_host_traced.err; exit 6; }
cd $R
python3 tools/host_overlap.py $O/trace $O/host_overlap.json || exit 7
