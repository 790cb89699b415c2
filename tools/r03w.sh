# round-3 GPU step w: C5 V-chunk length (build knob HHMM_VS_CHUNK) and C2's oracle check before / after the timed steps
mkdir -p gpurun_out/r03w
L=gsoc17-hhmm_amd/lib/libhhmm.so; V=gsoc17-hhmm_amd/lib/variants
timeout -k 10 300 python -u tools/ab_workload.py --workload c5 --rounds 7 --steps 2 vs512=$L vs256=$V/libhhmm_vs256.so vs1024=$V/libhhmm_vs1024.so > gpurun_out/r03w/c5.log 2>&1 || exit 3
for i in 1 2; do
  for w in after before; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --check-at $w > gpurun_out/r03w/c2_${w}_$i.json 2> gpurun_out/r03w/c2_${w}_$i.err || exit 4
  done
done
