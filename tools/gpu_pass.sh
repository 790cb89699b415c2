#!/bin/bash
# One GPU pass (via gpurun): optional new test files first, then an optional
# probe command, then the whole GPU suite + smoke.  Stops at the first failure;
# logs under gpurun_out/TAG/.
# Usage: tools/gpu_pass.sh TAG "<new test files or ''>" "<probe command or ''>" [suite]
set -o pipefail
TAG=$1; NEW=$2; PROBE=$3; SUITE=$4
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ -n "$NEW" ]; then
  timeout -k 10 400 python -u -m pytest $NEW -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
      > $O/new_tests.log 2>&1 || { echo "new tests rc=$?"; tail -30 $O/new_tests.log; exit 1; }
  echo "new tests ok: $(tail -1 $O/new_tests.log)"
fi
if [ -n "$PROBE" ]; then
  timeout -k 10 500 $PROBE > $O/probe.log 2>&1 || { echo "probe rc=$?"; tail -30 $O/probe.log; exit 2; }
  echo "probe ok"; grep -v amdgpu.ids $O/probe.log | tail -12
fi
if [ "$SUITE" = "suite" ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
      -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "suite rc=$?"; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 3; }
  echo "suite: $(tail -1 $O/pytest.log)"
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 4; }
  echo "smoke ok"
fi
