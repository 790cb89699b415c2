# round-3 GPU step af: smoke (now checks the library's source hash on the box) and the default bench line
mkdir -p gpurun_out/r03af
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03af/smoke.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03af/c2.json 2> gpurun_out/r03af/c2.err || exit 4
