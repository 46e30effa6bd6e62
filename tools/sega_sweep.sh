#!/bin/bash
# Same-box sweep of the first-level reduction segment count (MI_MSM_SEGA_LOG) for split-mode G1 MSMs.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sweep
for rep in 1 2; do
  for cfg in "MI_MSM_SEGA_LOG=20" "MI_MSM_SEGA_LOG=18" "MI_MSM_SEGA_LOG=19" "MI_MSM_SEGA_LOG=21" "MI_MSM_SPLIT=0"; do
    env $cfg timeout -k 10 200 python -u tools/msm_bench.py --log-rows 26 --reps 3 --query 0 > gpurun_out/sweep/s.log 2>&1
    echo "$cfg #$rep: $(tail -1 gpurun_out/sweep/s.log)"
  done
done
