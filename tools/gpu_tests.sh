#!/bin/bash
# Runs on the GPU box (via gpurun): the GPU test suite (or the test files given
# after TAG) under one time limit, then smoke(); logs under gpurun_out/TAG/.
# Usage: tools/gpu_tests.sh TAG [pytest targets ...]
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
TARGETS=${@:-tests}
timeout -k 10 900 python -u -m pytest $TARGETS -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> $O/pytest.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 4
