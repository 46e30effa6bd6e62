#!/bin/bash
# round 5, eighth GPU call: parity with every chunk-tree level counted in the plan readback (and L1 = 4), then the
# Winning-PoSt leg over chunk sizes L0 and tree fan-ins L1
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c8
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "boolean or window_table or random or split or glv" > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
MI_MSM_L1=4 timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "boolean or window_table" tests/test_gpu_post.py -k "boolean or window_table or winning" > $O/tests_l1_4.log 2>&1
rc=$?
tail -2 $O/tests_l1_4.log
[ $rc -eq 0 ] || exit $rc
W="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 20"
for v in base l1_4 l0_32 l0_32_l1_4 l0_16_l1_4 l0_16_l1_8 base2; do
  case $v in l1_4) E="MI_MSM_L1=4";; l0_32) E="MI_MSM_L0=32";; l0_32_l1_4) E="MI_MSM_L0=32 MI_MSM_L1=4";; l0_16_l1_4) E="MI_MSM_L0=16 MI_MSM_L1=4";; l0_16_l1_8) E="MI_MSM_L0=16 MI_MSM_L1=8";; *) E="X=1";; esac
  env $E timeout -k 10 300 $W > $O/win_$v.json 2> $O/win_$v.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$O/win_$v.json')); w=d['winning_post_32gib']; print('$v', round(w['latency_ms_median'],2), round(w['latency_ms_min'],2), w['verified'], w['device_ms_per_proof'])"
done
timeout -k 10 900 python3 -u -m pytest -x -q -s --timeout 800 --timeout-method thread tests/test_gpu_post.py -k "64gib" > $O/test_64gib.log 2>&1
rc=$?
grep "window-post-64\|passed\|failed" $O/test_64gib.log | tail -12
exit $rc
