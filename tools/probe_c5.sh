set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/probe; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 python -u $R/bench.py --steps 3 --warmup 1 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; exit 1; }; }
run c5_vit_states --workload c5 --pars zstar_t,logp_zstar --flags 16
run c5_logp_states --workload c5 --pars logp_zstar --flags 16
run c5_vit_lanes --workload c5 --pars zstar_t,logp_zstar --flags 8
run c5 --workload c5
