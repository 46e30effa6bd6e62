#!/bin/bash
# round 5, sixth GPU call: parity (window tables G1 + G2, balanced bit rows), 2^20 timelines at c = 16 / 20, and the
# Winning-PoSt leg with / without window tables
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c6
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_groth16.py > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for t in 16 20; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/tr_$t -o run -- python3 tools/msm_bench.py --log-rows 20 --reps 20 --table $t > $O/msm_$t.txt 2>&1 || exit 1
  tail -1 $O/msm_$t.txt
  python3 tools/msm_timeline.py /tmp/tr_$t/run_results.db --reps 10 > $O/timeline_$t.md
  head -16 $O/timeline_$t.md
done
W="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 20"
for v in wt g1only nowt; do
  case $v in nowt) E="MI_MSM_WT_MAX_LOG=0";; g1only) E="MI_PROVE_B1_LANE=0";; *) E="";; esac
  env $E timeout -k 10 300 $W > $O/win_$v.json 2> $O/win_$v.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$O/win_$v.json')); w=d['winning_post_32gib']; print('$v', w['latency_ms_median'], w['latency_ms_min'], w['verified'], w['device_ms_per_proof'])"
done
