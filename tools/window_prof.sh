#!/bin/bash
# Kernel trace of the 32 GiB Window-PoSt leg (GPU witness + proof per partition) with prove_lanes=1 (both
# lanes' work on one stream, so each kernel runs alone), then tools/winning_timeline.py over the last partition.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-winpost}
mkdir -p gpurun_out/$T
B=(python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --uniform-steps 0 --winning-log-nodes 0 --post-reps 2 --post-share-groups "" --tune prove_lanes=1)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/trace -o run -- "${B[@]}" > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/winning_timeline.py gpurun_out/$T/trace/run_results.db --reps 1 --md > gpurun_out/$T/timeline.md
cat gpurun_out/$T/timeline.md
