#!/bin/bash
# round 5, fifteenth GPU call: the whole GPU suite and smoke() as the driver runs them, then the refreshed
# Winning-PoSt breakdown trace (kernel + HIP runtime traces; databases kept in /tmp)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c15
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -2 $O/smoke.log
B="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 10"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d /tmp/win15 -o run -- $B > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
python3 tools/winning_timeline.py /tmp/win15/run_results.db --md > $O/timeline.md
python3 tools/call_timeline.py /tmp/win15/run_results.db --kernels --min-ms 0.2 > $O/call.txt
cat $O/timeline.md
grep "^stream\|gaps\|host tid" $O/call.txt
