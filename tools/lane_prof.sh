#!/bin/bash
# One profiled bench of the main path (2^26, config 3) for the lane timeline (tools/lane_timeline.py), plus
# unprofiled bench lines with both lanes and with MI_PROVE_LANES=1 (serial: per-phase device time).
#   bash tools/lane_prof.sh <tag> [extra bench args]
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-lane}; shift || true
B="python3 bench.py --steps 3 --warmup 1 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --config4-log-rows 0 --sdr-log-labels 0 --stacked-log-nodes 0 --post-sectors 0 --winning-log-nodes 0 --uniform-steps 0 $*"
mkdir -p gpurun_out/$T
timeout -k 10 300 $B > gpurun_out/$T/two_lanes.json 2> gpurun_out/$T/two_lanes.err
MI_PROVE_LANES=1 timeout -k 10 300 $B > gpurun_out/$T/one_lane.json 2> gpurun_out/$T/one_lane.err
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$T/trace -o run -- $B > gpurun_out/$T/trace.json 2> gpurun_out/$T/trace.err
echo done
