#!/bin/bash
# rocprofv3 evidence for the round's bench line (per-round tag): kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md).  The profiled command is the bench's main
# path only (the bench's default warm-up and timed proofs, pipelined as in the bench line, then the standalone MSM): no CPU baseline, device-resident, tree C or
# config-4 legs, so the launch order matches tools/profile_summary.py's reconstruction.
#   bash tools/prof_round.sh [tag]       then: python tools/profile_summary.py --tag <tag> ...
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-r2}
B="python3 bench.py --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --config4-log-rows 0 --sdr-log-labels 0 --stacked-log-nodes 0 --post-sectors 0 --winning-log-nodes 0 --uniform-steps 0 --params-roundtrip 0"
mkdir -p gpurun_out
echo "$B" > gpurun_out/${T}_command.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_trace -o run -- $B > gpurun_out/${T}_trace.json 2> gpurun_out/${T}_trace.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch -o run -- $B > gpurun_out/${T}_fetch.json 2> gpurun_out/${T}_fetch.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write -o run -- $B > gpurun_out/${T}_write.json 2> gpurun_out/${T}_write.err
echo done
