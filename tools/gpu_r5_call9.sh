#!/bin/bash
# round 5, ninth GPU call: Winning-PoSt call timeline (kernel + HIP runtime traces; databases kept in /tmp)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c9
mkdir -p $O
B="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 10"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d /tmp/win9 -o run -- $B > $O/bench.json 2> $O/bench.err || exit 1
python3 tools/winning_timeline.py /tmp/win9/run_results.db --md > $O/timeline.md
python3 tools/call_timeline.py /tmp/win9/run_results.db --kernels --min-ms 0.2 > $O/call.txt
cat $O/timeline.md
head -150 $O/call.txt
