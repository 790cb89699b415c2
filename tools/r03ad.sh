# round-3 GPU step ad: phased sweep workgroup size (HHMM_PROBE_FB_WAVES applies to vfb_kernel's launch shape)
mkdir -p gpurun_out/r03ad
timeout -k 10 400 python -u tools/ab_sched.py --rounds 7 --steps 3 vfb vfb@HHMM_PROBE_FB_WAVES=1 vfb@HHMM_PROBE_FB_WAVES=2 vfb@HHMM_PROBE_FB_WAVES=3 > gpurun_out/r03ad/ab.json 2> gpurun_out/r03ad/ab.err || exit 3
