#!/bin/bash
# Winning-PoSt latency under MSM knobs (window size MI_MSM_C, split mode, one lane): one bench process per
# setting, only the Winning leg after a tiny main leg; prints "setting latency_ms_median".
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wsweep
B="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 20"
run() {
    local tag=$1; shift
    env "$@" timeout -k 10 180 $B > gpurun_out/wsweep/$tag.json 2> gpurun_out/wsweep/$tag.err || return 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/wsweep/$tag.json').read().strip().splitlines()[-1])['winning_post_32gib']; print('$tag', round(d['latency_ms_median'],2), round(d['latency_ms_min'],2), d['verified'])"
}
run default MI_X=0 || exit 1
for c in 12 13 14 15 16; do run c$c MI_MSM_C=$c || exit 1; done
run nosplit MI_MSM_SPLIT=0 || exit 1
run onelane MI_PROVE_LANES=1 || exit 1
run default2 MI_X=0 || exit 1
