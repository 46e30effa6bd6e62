#!/bin/bash
# round-4: full -m gpu suite after the onesweep-for-small-sorts and lane-parallel phase-A Poseidon changes, then
# the Winning-PoSt trace and the bench legs
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests6.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/r04_gpu_tests6.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/winning_prof.sh win2 || exit 1
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --config4-log-rows 0 --tree-log-nodes 0 --sdr-log-labels 0 --uniform-steps 0 > gpurun_out/r04_bench_legs2.json 2> gpurun_out/r04_bench_legs2.err
echo "bench rc=$?"; tail -3 gpurun_out/r04_bench_legs2.err
