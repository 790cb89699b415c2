# round-3 GPU step s: C5 / N2 with the side pass on a high-priority stream (HHMM_PROBE_SIDE_PRIO)
mkdir -p gpurun_out/r03s
L=gsoc17-hhmm_amd/lib/libhhmm.so
timeout -k 10 300 python -u tools/ab_workload.py --workload c5 --rounds 7 --steps 2 base=$L prio=$L@HHMM_PROBE_SIDE_PRIO=1 > gpurun_out/r03s/c5.log 2>&1 || exit 3
