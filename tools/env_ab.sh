#!/bin/bash
# Same-box A/B of an environment knob in the full prove: bash tools/env_ab.sh VAR "v1 v2" [reps]
# (each value runs the Groth16 GPU tests once -- TESTK overrides the -k filter, then bench.py alternates the values)
cd "$GRAFT_REPO_ROOT" || exit 1
VAR=$1; VALS=$2; REPS=${3:-2}
mkdir -p gpurun_out/env
for v in $VALS; do
  env "$VAR=$v" timeout -k 10 300 python -u -m pytest tests/test_gpu_groth16.py tests/test_gpu_kernels.py -x -q -k "${TESTK:-g2 or groth16}" --timeout 200 --timeout-method thread > gpurun_out/env/t_$v.log 2>&1 || { echo "$VAR=$v tests FAILED: $(tail -3 gpurun_out/env/t_$v.log)"; exit 1; }
  echo "$VAR=$v tests: $(tail -1 gpurun_out/env/t_$v.log)"
done
for rep in $(seq 1 "$REPS"); do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-device-resident --steps 6 --warmup 1 \
        --msm-reps 1 --tree-log-nodes 0 --config4-log-rows 0 > gpurun_out/env/b_${v}_$rep.json 2> gpurun_out/env/b_${v}_$rep.err || { echo "bench failed"; exit 1; }
    echo "$VAR=$v #$rep: $(python3 -c "
import json; b = json.load(open('gpurun_out/env/b_${v}_$rep.json')); t = b['timers_ms']; s = b['steps']
print(round(b['value'] / 1e6, 2), 'Mc/s', round(b['ms_per_step'], 1), 'ms/proof; msm_g2', round(t['msm_g2'] / s, 1), 'accum_g2', round(t['accum_g2'] / s, 1), 'msm_g1', round(t['msm_g1'] / s, 1), 'sort', round(t['sort'] / s, 1), 'GB', b.get('device_gb_after_setup'), 'srs_s', round(b['setup_s']['srs'], 1), 'verified', b['verified'])")"
  done
done
