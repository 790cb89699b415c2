# round-3 GPU step y: bench.py --gpus 2 rehearsal on the one-GPU box (both ranks on GPU 0, gloo), then --gpus 1
mkdir -p gpurun_out/r03y
HHMM_BENCH_BACKEND=gloo HHMM_BENCH_SHARE_DEVICES=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r03y/g2.json 2> gpurun_out/r03y/g2.err || exit 3
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03y/g1.json 2> gpurun_out/r03y/g1.err || exit 4
