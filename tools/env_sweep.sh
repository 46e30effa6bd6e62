#!/bin/bash
# Same-box sweep of MSM tuning knobs read from the environment (no rebuild):
#   MI_MSM_L0 (entries per level-0 chunk), MI_MSM_SEGA_LOG (first-level reduction segments).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sweep
Q=${1:-0}
for rep in 1 2; do
  for cfg in "MI_MSM_L0=64" "MI_MSM_L0=32" "MI_MSM_L0=128" "MI_MSM_SEGA_LOG=19" "MI_MSM_SEGA_LOG=21"; do
    env $cfg timeout -k 10 200 python -u tools/msm_bench.py --log-rows 26 --reps 3 --query $Q > gpurun_out/sweep/s.log 2>&1
    echo "q$Q $cfg #$rep: $(tail -1 gpurun_out/sweep/s.log)"
  done
done
