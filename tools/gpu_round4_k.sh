#!/bin/bash
# round-4 final, part 2: the default bench line (the driver's command) and the one-lane trace of a 2^26 proof
mkdir -p gpurun_out
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_bench_default.json 2> gpurun_out/r04_bench_default.err
echo "bench rc=$?"; grep "^\[bench\]" gpurun_out/r04_bench_default.err | tail -4
bash tools/lane_prof1.sh r04_lane1
