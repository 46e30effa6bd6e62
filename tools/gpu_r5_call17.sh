#!/bin/bash
# round 5, seventeenth GPU call: witness parity with the latency-form Fr products in the Poseidon lanes, then the
# Winning-PoSt, stacked-PoRep and Window-PoSt witness legs
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c17
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stacked.py tests/test_gpu_post.py tests/test_gpu_poseidon.py -k "not 64gib" > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
W="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 20"
for v in a b; do
  timeout -k 10 300 $W > $O/win_$v.json 2> $O/win_$v.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$O/win_$v.json')); w=d['winning_post_32gib']; print('$v', round(w['latency_ms_median'],2), round(w['latency_ms_min'],2), w['verified'], w['device_ms_per_proof'])"
done
