#!/bin/bash
# Same-box A/B of the lane configurations and the fused QAP pass at 2^26 (config 3), two runs each,
# interleaved: default two lanes / aux lane high priority / main lane high priority / one lane
# (MI_PROVE_LANES=1) / unfused QAP division (MI_QAP_FUSED=0).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab2
B="python3 bench.py --steps 4 --warmup 1 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --config4-log-rows 0 --sdr-log-labels 0 --stacked-log-nodes 0"
for rep in 1 2; do
  for cfg in default aux_hi main_hi one_lane qap_unfused; do
    case $cfg in
      default) E="" ;;
      aux_hi) E="MI_LANE_PRIO=aux" ;;
      main_hi) E="MI_LANE_PRIO=main MI_BENCH_PRIORITY=1" ;;
      one_lane) E="MI_PROVE_LANES=1" ;;
      qap_unfused) E="MI_QAP_FUSED=0" ;;
    esac
    env $E timeout -k 10 300 $B > gpurun_out/ab2/$cfg.$rep.json 2> gpurun_out/ab2/$cfg.$rep.err
    python3 -c "import json; b=json.load(open('gpurun_out/ab2/$cfg.$rep.json')); print('$cfg', $rep, round(b['ms_per_step'],1), 'ms', b['verified'], round(b['timers_ms']['ntt']/max(1,b['steps']),2), 'ms ntt/proof')"
  done
done
