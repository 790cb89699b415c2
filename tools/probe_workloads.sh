set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/probe; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 python -u $R/bench.py --steps 3 --warmup 1 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; exit 1; }; }
run c5_fb --workload c5 --pars loglik,gamma_tk
run c5_vit_states --workload c5 --pars zstar_t,logp_zstar --flags 16
run c5_vit_lanes --workload c5 --pars zstar_t,logp_zstar --flags 8
run c5_logp_states --workload c5 --pars logp_zstar --flags 16
run c5_logp_lanes --workload c5 --pars logp_zstar --flags 8
run c3_loglik --workload c3 --pars loglik
run c3_gamma --workload c3 --pars loglik,gamma_tk
run c3_vit --workload c3 --pars zstar_t,logp_zstar
run c4_gamma --workload c4 --pars loglik,gamma_tk
run c4_ffbs --workload c4 --pars z_ffbs
