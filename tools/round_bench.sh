#!/bin/bash
# Runs on the GPU box (via gpurun): the judged default bench line (C2) and
# every evidence workload, each with its CPU baseline, under its own time
# limit; stops at the first failure.
# Usage: tools/round_bench.sh TAG  -> gpurun_out/rb_TAG/{c2,c1,c3,c4,c5,n1,n2,f1,c2-host}.json
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rb_$TAG
mkdir -p $O
run() {
  name=$1; shift
  timeout -k 10 240 python -u $R/bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name rc=$?"; exit 1; }
  echo "ok $name"
}
run c2 --steps 20 --warmup 5
for w in c1 c3 c4 c5 n1 n2 f1; do
  run $w --workload $w --steps 5 --warmup 2
done
run c2-host --workload c2-host --steps 3 --warmup 1
exit 0
