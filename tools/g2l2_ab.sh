#!/bin/bash
# Same-box A/B of the G2 bucket reduction (MI_G2_L2=0 running sums, 1 second-level MSM): standalone
# G2 MSM at 2^26 rows, then the full prove bench.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g2l2
for rep in 1 2; do
  for m in 0 1; do
    MI_G2_L2=$m timeout -k 10 200 python -u tools/msm_bench.py --log-rows 26 --reps 3 --query 4 > gpurun_out/g2l2/m.log 2>&1
    echo "msm L2=$m #$rep: $(tail -1 gpurun_out/g2l2/m.log)"
  done
done
for m in 0 1 0 1; do
  MI_G2_L2=$m timeout -k 10 300 python -u bench.py --no-cpu-baseline --msm-reps 1 > gpurun_out/g2l2/b.json 2> gpurun_out/g2l2/b.err
  echo "prove L2=$m: $(python3 -c "import json; b=json.load(open('gpurun_out/g2l2/b.json')); print(round(b['value']/1e6,2), 'Mc/s', round(b['ms_per_step'],1), 'ms', b['timers_ms']['msm_g2'], b['timers_ms']['accum_g2'])")"
done
