set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
B="python3 bench.py --steps 1 --warmup 1 --msm-reps 1 --no-cpu-baseline"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1_trace -o run -- $B > gpurun_out/r1_trace.json 2> gpurun_out/r1_trace.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r1_fetch -o run -- $B > gpurun_out/r1_fetch.json 2> gpurun_out/r1_fetch.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r1_write -o run -- $B > gpurun_out/r1_write.json 2> gpurun_out/r1_write.err
echo done
