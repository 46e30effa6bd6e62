#!/bin/bash
# Same-box A/B of library builds in the full prove: build/var/lib_<v>.so for each variant.
# The variants listed in $TEST_VARIANTS first run the MSM kernel + Groth16 GPU tests once
# (correctness gate), then bench.py alternates the variants $REPS times so box drift shows up.
#   bash tools/prove_ab.sh "a b" [reps]
cd "$GRAFT_REPO_ROOT" || exit 1
V=${1:-"a b"}; REPS=${2:-2}
mkdir -p gpurun_out/ab
for v in ${TEST_VARIANTS:-}; do
  FILGPU_LIB=crypto3-fil-proofs_amd/build/var/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py \
      tests/test_gpu_groth16.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/t_$v.log 2>&1 || {
    echo "$v tests FAILED: $(tail -3 gpurun_out/ab/t_$v.log)"; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/ab/t_$v.log)"
done
for rep in $(seq 1 "$REPS"); do
  for v in $V; do
    FILGPU_LIB=crypto3-fil-proofs_amd/build/var/lib_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline \
        --no-device-resident --steps ${STEPS:-5} --warmup 1 --msm-reps 2 ${BENCH_ARGS:-} \
        > gpurun_out/ab/b_${v}_$rep.json 2> gpurun_out/ab/b_${v}_$rep.err || { echo "$v bench FAILED"; exit 1; }
    echo "$v#$rep: $(python3 -c "
import json; b = json.load(open('gpurun_out/ab/b_${v}_$rep.json')); t = b['timers_ms']; s = b['steps']
print(round(b['value'] / 1e6, 2), 'Mc/s', round(b['ms_per_step'], 1), 'ms/proof; accum_g1', round(t['accum_g1'] / s, 1),
      'accum_g2', round(t['accum_g2'] / s, 1), 'msm_g1', round(t['msm_g1'] / s, 1), 'ntt', round(t['ntt'] / s, 1),
      'sort', round(t['sort'] / s, 1), '| G1 MSM', round(b['msm_g1_mpoints_per_s'], 1), 'Mpts/s; verified', b['verified'])")"
  done
done
