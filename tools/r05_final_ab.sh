#!/bin/bash
# Round-5 final build, both passes in one call (via gpurun): the GPU suite +
# smoke, then pass A (tools/r05_final_a.sh: the judged C2 command under
# rocprofv3, C2 PMC, per-workload PMC), then every bench line
# (tools/round_bench.sh).  The bench lines of this call carry no PMC fields
# (bench_traffic.json is rewritten from pass A afterwards, on the CPU side).
# Usage: tools/r05_final_ab.sh TAG
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
bash tools/r05_final_a.sh $TAG || exit 3
cd $R
bash tools/round_bench.sh $TAG || exit 4
