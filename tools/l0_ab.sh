#!/bin/bash
# Same-box A/B of the level-0 chunk length in the full prove (MI_MSM_L0).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/l0
for L in 64 128 256 64 128 256; do
  MI_MSM_L0=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --msm-reps 1 > gpurun_out/l0/b.json 2> gpurun_out/l0/b.err
  echo "prove L0=$L: $(python3 -c "import json; b=json.load(open('gpurun_out/l0/b.json')); print(round(b['value']/1e6,2), 'Mc/s', round(b['ms_per_step'],1), 'ms', round(b['msm_g1_mpoints_per_s'],1))")"
done
