#!/bin/bash
# Winning-PoSt latency against the MSM window size (MI_MSM_C) on the plain (unsplit) path of 2^18-2^19-point MSMs
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/csweep
B="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 20"
for c in def 12 13 14 15 17 def; do
    if [ $c = def ]; then timeout -k 10 180 $B > gpurun_out/csweep/$c.json 2> gpurun_out/csweep/$c.err || exit 1
    else MI_MSM_C=$c timeout -k 10 180 $B > gpurun_out/csweep/$c.json 2> gpurun_out/csweep/$c.err || exit 1; fi
    python3 -c "import json; d=json.loads(open('gpurun_out/csweep/$c.json').read().strip().splitlines()[-1])['winning_post_32gib']; print('c=$c', round(d['latency_ms_median'],2), round(d['latency_ms_min'],2), d['verified'])"
done
