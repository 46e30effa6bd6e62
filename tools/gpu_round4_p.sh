# round-4 final: the default bench line (no flags: the driver's N=1 command shape)
mkdir -p gpurun_out
timeout -k 10 900 python3 bench.py > gpurun_out/r04_bench_default2.json 2> gpurun_out/r04_bench_default2.err
echo "bench rc=$?"; grep "^\[bench\]" gpurun_out/r04_bench_default2.err | tail -3
