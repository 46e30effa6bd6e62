#!/bin/bash
# Same-box A/B of the aux-lane MSM order in the full prove (MI_AUX_ORDER).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lane
for o in l_first b_first l_first b_first; do
  MI_AUX_ORDER=$o timeout -k 10 300 python -u bench.py --no-cpu-baseline --msm-reps 1 > gpurun_out/lane/b.json 2> gpurun_out/lane/b.err
  echo "prove $o: $(python3 -c "import json; b=json.load(open('gpurun_out/lane/b.json')); print(round(b['value']/1e6,2), 'Mc/s', round(b['ms_per_step'],1), 'ms')")"
done
