# round-3 GPU step l: which of the wait restructurings cost time (asm register copies, loop-entry drains)
mkdir -p gpurun_out/r03l
V=gsoc17-hhmm_amd/lib/variants
timeout -k 10 500 python -u tools/ab_sched.py --lib rc0=$V/libhhmm_rc0.so --lib dr0=$V/libhhmm_dr0.so --lib rc0dr0=$V/libhhmm_rc0dr0.so --lib base=$V/libhhmm_base.so rc0:vfb dr0:vfb rc0dr0:vfb base:vfb rc0dr0:two base:two > gpurun_out/r03l/ab_sched.json 2> gpurun_out/r03l/ab_sched.err || exit 4
