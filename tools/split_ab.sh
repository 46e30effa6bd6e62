#!/bin/bash
# Same-box A/B of the split-mode G1 MSM (MI_MSM_SPLIT=0 plain, 1 default) in the full prove + G1 MSM.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/split
for m in 0 1 0 1; do
  MI_MSM_SPLIT=$m timeout -k 10 300 python -u bench.py --no-cpu-baseline --msm-reps 2 > gpurun_out/split/b$m.json 2> gpurun_out/split/b$m.err
  echo "split=$m: $(python3 -c "import json; b=json.load(open('gpurun_out/split/b$m.json')); print(round(b['value']/1e6,2), 'Mc/s', round(b['ms_per_step'],1), 'ms; msm', round(b['msm_g1_mpoints_per_s'],1), 'Mpts/s')")"
done
