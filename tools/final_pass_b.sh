#!/bin/bash
# Final build, pass B (via gpurun): the whole GPU suite + smoke, then
# every bench line (tools/round_bench.sh: C2 as the driver runs it, and the
# evidence workloads with their CPU baselines), once profiles/bench_traffic.json
# holds pass A's PMC of this build.  Stops at the first failure.
# Usage: tools/final_pass_b.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "suite rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 2; }
echo "smoke ok"
bash tools/round_bench.sh $TAG || exit 3
