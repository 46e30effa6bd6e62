#!/bin/bash
# round-4: GPU tests from test_gpu_groth16 on (range shares, OOM fallback, two 32 GiB keys, Winning PoSt), then a
# bench run of the main leg + Winning-PoSt + Window-PoSt legs (latency groups computing H once)
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_groth16.py tests/test_gpu_memory.py tests/test_gpu_post.py tests/test_gpu_poseidon.py tests/test_gpu_scale.py tests/test_gpu_sdr.py tests/test_gpu_stacked.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests4.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/r04_gpu_tests4.log; grep "two-keys" gpurun_out/r04_gpu_tests4.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --config4-log-rows 0 --stacked-log-nodes 0 --tree-log-nodes 0 --sdr-log-labels 0 > gpurun_out/r04_bench_legs.json 2> gpurun_out/r04_bench_legs.err
echo "bench rc=$?"; tail -3 gpurun_out/r04_bench_legs.err
