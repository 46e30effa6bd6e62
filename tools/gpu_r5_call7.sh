#!/bin/bash
# round 5, seventh GPU call: parity after the shared-plan tree fix (every lane layout of the 32 GiB Winning PoSt
# byte-identical), then Winning-PoSt and 2^20 variants (window bits, bit-sum fan-in)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c7
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_groth16.py tests/test_gpu_post.py > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for g in 4 8 16; do
  MI_MSM_BS_G0=$g timeout -k 10 200 python3 tools/msm_bench.py --log-rows 20 --reps 50 --table 20 2>&1 | grep "G1 MSM" | sed "s/^/G0=$g /" || exit 1
done
W="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 20"
for v in wt c20 b1l0 nowt wt2; do
  case $v in nowt) E="MI_MSM_WT_MAX_LOG=0";; c20) E="MI_MSM_WT_C=20";; b1l0) E="MI_PROVE_B1_LANE=0";; *) E="";; esac
  env $E timeout -k 10 300 $W > $O/win_$v.json 2> $O/win_$v.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$O/win_$v.json')); w=d['winning_post_32gib']; print('$v', round(w['latency_ms_median'],2), round(w['latency_ms_min'],2), w['verified'], w['device_ms_per_proof'])"
done
