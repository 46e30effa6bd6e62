#!/bin/bash
# round 5, tenth GPU call: parity after the launch trimming (binary-search chunk / partial owners, fused init,
# one-copy plan readback, division-free level counts), then 2^20 and Winning-PoSt timing and a Winning trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c10
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_groth16.py tests/test_gpu_post.py -k "not 64gib" > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/msm_bench.py --log-rows 20 --reps 50 --table 20 2>&1 | grep "G1 MSM" || exit 1
W="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 20"
for v in a b; do
  timeout -k 10 300 $W > $O/win_$v.json 2> $O/win_$v.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$O/win_$v.json')); w=d['winning_post_32gib']; print('$v', round(w['latency_ms_median'],2), round(w['latency_ms_min'],2), w['verified'], w['device_ms_per_proof'])"
done
B="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 10"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d /tmp/win10 -o run -- $B > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
python3 tools/winning_timeline.py /tmp/win10/run_results.db --md > $O/timeline.md
python3 tools/call_timeline.py /tmp/win10/run_results.db --kernels --min-ms 0.2 > $O/call.txt
cat $O/timeline.md
grep "^stream\|gaps\|host tid" $O/call.txt
