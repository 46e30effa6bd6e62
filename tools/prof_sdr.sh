#!/bin/bash
# rocprofv3 evidence for the SDR label kernel: kernel trace + stats of tools/sdr_bench.py,
# then FETCH_SIZE and WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md), each under its own limit.
#   bash tools/prof_sdr.sh [tag]
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r02_sdr}
B="python3 tools/sdr_bench.py --no-cpu-baseline"
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_trace -o run -- $B > gpurun_out/${T}_trace.json 2> gpurun_out/${T}_trace.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch -o run -- $B > gpurun_out/${T}_fetch.json 2> gpurun_out/${T}_fetch.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write -o run -- $B > gpurun_out/${T}_write.json 2> gpurun_out/${T}_write.err
echo done
