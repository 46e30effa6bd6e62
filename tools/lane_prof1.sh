#!/bin/bash
# Kernel trace of the main path with prove_lanes=1 (both lanes' work serialised on one stream): the
# per-kernel device time of one proof without the other lane's kernels beside it (tools/lane_timeline.py).
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-lane1}; shift || true
B="python3 bench.py --steps 3 --warmup 1 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --config4-log-rows 0 --sdr-log-labels 0 --stacked-log-nodes 0 --post-sectors 0 --winning-log-nodes 0 --uniform-steps 0 $*"
mkdir -p gpurun_out/$T
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$T/trace -o run -- $B --tune prove_lanes=1 > gpurun_out/$T/trace.json 2> gpurun_out/$T/trace.err
echo done
