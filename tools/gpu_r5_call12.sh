#!/bin/bash
# round 5, twelfth GPU call: parity with the uncapped bit-row kernels (G2 lane pairs in registers), Winning PoSt and
# the 2^20 MSM
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c12
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_groth16.py tests/test_gpu_post.py -k "not 64gib" > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
W="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 20"
for v in a b; do
  timeout -k 10 300 $W > $O/win_$v.json 2> $O/win_$v.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$O/win_$v.json')); w=d['winning_post_32gib']; print('$v', round(w['latency_ms_median'],2), round(w['latency_ms_min'],2), w['verified'], w['device_ms_per_proof'])"
done
for t in 20 16; do
  timeout -k 10 200 python3 tools/msm_bench.py --log-rows 20 --reps 50 --table $t 2>&1 | grep "G1 MSM" || exit 1
done
MI_MSM_BS_SEG_LOG=17 timeout -k 10 200 python3 tools/msm_bench.py --log-rows 20 --reps 50 --table 20 2>&1 | grep "G1 MSM" | sed "s/^/seg17 /" || exit 1
