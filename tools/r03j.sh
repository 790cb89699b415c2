# round-3 GPU step j: the phased sweep as the C2 default -- whole GPU suite, C2 bench, kernel trace + PMC; C5 tie-list A/B
mkdir -p gpurun_out/r03j
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03j/pytest.log 2>&1
rc=$?; echo PYTEST_EXIT $rc >> gpurun_out/r03j/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03j/c2.json 2> gpurun_out/r03j/c2.err || exit 4
timeout -k 10 400 python -u tools/ab_workload.py --workload c5 head=gsoc17-hhmm_amd/lib/libhhmm.so tieinl=gsoc17-hhmm_amd/lib/variants/libhhmm_tieinl.so --rounds 5 --steps 2 > gpurun_out/r03j/ab_c5.log 2>&1 || exit 5
bash tools/profile_box.sh r03j > gpurun_out/r03j/prof.log 2>&1
echo PROF_EXIT $? >> gpurun_out/r03j/prof.log
