# round-3 GPU step u: C5 forward-backward T-chunk length below 512 (high-priority side stream)
mkdir -p gpurun_out/r03u
L=gsoc17-hhmm_amd/lib/libhhmm.so
timeout -k 10 300 python -u tools/ab_workload.py --workload c5 --rounds 7 --steps 2 auto=$L cl64=$L#0x600 cl128=$L#0x700 cl256=$L#0x800 > gpurun_out/r03u/c5.log 2>&1 || exit 3
