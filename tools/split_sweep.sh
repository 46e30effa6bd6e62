#!/bin/bash
# Split-mode threshold (MI_MSM_SPLIT_MIN, log2 points) against the Winning-PoSt latency and the 2^20 G1 MSM
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ssweep
B="python3 bench.py --steps 2 --warmup 1 --log-rows 21 --msm-reps 2 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 20"
for lg in ${SPLIT_SWEEP:-16 19 20 21 16}; do
    if [ "$lg" = def ]; then
        timeout -k 10 240 $B > gpurun_out/ssweep/s$lg.json 2> gpurun_out/ssweep/s$lg.err || exit 1
    else
        MI_MSM_SPLIT_MIN=$lg timeout -k 10 240 $B > gpurun_out/ssweep/s$lg.json 2> gpurun_out/ssweep/s$lg.err || exit 1
    fi
    python3 -c "import json; d=json.loads(open('gpurun_out/ssweep/s$lg.json').read().strip().splitlines()[-1]); w=d['winning_post_32gib']; m=d['config2_micro']; print('split_min 2^$lg', 'winning', round(w['latency_ms_median'],2), 'msm2^20', round(m['msm_g1_2e20_ms'],3), 'ms', 'prove2^21', round(d['ms_per_step'],2))"
done
