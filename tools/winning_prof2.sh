#!/bin/bash
# Winning-PoSt latency leg under rocprofv3 with kernel, memory-copy and HIP runtime traces (host gaps between
# launches and synchronisations), for tools/winning_timeline.py and a per-stream look at one call.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-win3}; shift
mkdir -p gpurun_out/$T
B="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 10 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d gpurun_out/$T/trace -o run -- $B > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/winning_timeline.py gpurun_out/$T/trace/run_results.db --md > gpurun_out/$T/timeline.md
cat gpurun_out/$T/timeline.md
