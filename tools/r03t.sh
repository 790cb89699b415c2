# round-3 GPU step t: high-priority side stream as the default (C5, N2) and the C5 forward-backward T-chunk length
mkdir -p gpurun_out/r03t
L=gsoc17-hhmm_amd/lib/libhhmm.so
timeout -k 10 300 python -u tools/ab_workload.py --workload c5 --rounds 7 --steps 2 prio=$L noprio=$L@HHMM_PROBE_SIDE_PRIO=0 cl256=$L#0x800 cl1024=$L#0xA00 cl2048=$L#0xB00 > gpurun_out/r03t/c5.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/ab_workload.py --workload n1 --rounds 3 --steps 2 prio=$L noprio=$L@HHMM_PROBE_SIDE_PRIO=0 > gpurun_out/r03t/n1.log 2>&1 || exit 4
