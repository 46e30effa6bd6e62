#!/bin/bash
# round 5, thirteenth GPU call: the default bench line, then the round's rocprofv3 evidence (kernel trace + stats,
# FETCH_SIZE and WRITE_SIZE passes) summarised on the box into profiles/r05_summary.json; traces removed after
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c13
mkdir -p $O
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
tail -c 600 $O/bench.json
bash tools/prof_round.sh r05 || exit 1
python3 tools/profile_summary.py --tag r05 --trace gpurun_out/r05_trace --fetch gpurun_out/r05_fetch --write gpurun_out/r05_write --bench-json gpurun_out/r05_trace.json --command-file gpurun_out/r05_command.txt > $O/summary.txt 2>&1 || exit 1
cp profiles/r05_summary.json profiles/r05_kernel_stats.csv $O/
rm -rf gpurun_out/r05_trace gpurun_out/r05_fetch gpurun_out/r05_write
head -30 $O/summary.txt
