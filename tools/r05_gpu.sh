#!/bin/bash
# Round-5 GPU pass (via gpurun): the new GPU tests first, then the whole GPU
# suite + smoke, then the judged bench command twice -- once under
# rocprofv3 --kernel-trace --stats (one process: the JSON line and the kernel
# trace it produced), once plain.  Stops at the first failure.
# Usage: tools/r05_gpu.sh TAG [new test files...]
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
      > $O/new_tests.log 2>&1 || { echo "new tests rc=$?"; tail -30 $O/new_tests.log; exit 1; }
  echo "new tests ok"; tail -2 $O/new_tests.log
fi
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "suite rc=$?"; tail -40 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 3; }
echo "smoke ok"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_traced.json 2> $O/bench_traced.err \
    || { echo "traced bench rc=$?"; tail -20 $O/bench_traced.err; exit 4; }
echo "traced bench ok"
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
    || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 5; }
echo "bench ok"
exit 0
