#!/bin/bash
# round 5, fourth GPU call: window-table MSMs (parity first), then the 2^20 MSM and Winning-PoSt A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c4
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_groth16.py > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for t in -1 0 16 18 20; do
  timeout -k 10 200 python3 tools/msm_bench.py --log-rows 20 --reps 20 --table $t 2>&1 | grep -v "^W2026\|amdgpu.ids" | tail -2 || exit 1
done
MI_MSM_BITSUM=0 timeout -k 10 200 python3 tools/msm_bench.py --log-rows 20 --reps 20 --table 18 2>&1 | tail -1 || exit 1
W="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 20"
for v in wt nowt wt; do
  if [ $v = nowt ]; then E="MI_MSM_WT_MAX_LOG=0"; else E=""; fi
  env $E timeout -k 10 300 $W > $O/win_$v.json 2> $O/win_$v.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$O/win_$v.json')); w=d['winning_post_32gib']; print('$v', w['latency_ms_median'], w['latency_ms_min'], w['verified'], w['device_ms_per_proof'])"
done
