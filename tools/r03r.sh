# round-3 GPU step r: persistent / staggered phased-sweep probe (HHMM_PROBE_VFB_PERSIST) against the default
mkdir -p gpurun_out/r03r
timeout -k 10 400 python -u tools/ab_sched.py --rounds 7 --steps 3 vfb vfb@HHMM_PROBE_VFB_PERSIST=2/0 vfb@HHMM_PROBE_VFB_PERSIST=1/90 vfb@HHMM_PROBE_VFB_PERSIST=1/184 vfb@HHMM_PROBE_VFB_PERSIST=2/184 vfb@HHMM_PROBE_VFB_PERSIST=1/40 > gpurun_out/r03r/ab.json 2> gpurun_out/r03r/ab.err
