#!/bin/bash
# Round 5 same-box A/B of two library builds (build/var/lib_<v>.so): GPU correctness gate on the variants in
# $TEST_VARIANTS, then bench.py's main leg + uniform witness + Winning / Window PoSt alternated $REPS times.
#   bash tools/gpu_r5_ab.sh "old new" [reps]
cd "$GRAFT_REPO_ROOT" || exit 1
V=${1:-"old new"}; REPS=${2:-2}
mkdir -p gpurun_out/ab5
for v in ${TEST_VARIANTS:-}; do
  FILGPU_LIB=crypto3-fil-proofs_amd/build/var/lib_$v.so timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_kernels.py tests/test_gpu_groth16.py} \
      -x -q -k "${TESTK:-not nothing_excluded}" --timeout 300 --timeout-method thread > gpurun_out/ab5/t_$v.log 2>&1 || {
    echo "$v tests FAILED: $(tail -5 gpurun_out/ab5/t_$v.log)"; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/ab5/t_$v.log)"
done
for rep in $(seq 1 "$REPS"); do
  for v in $V; do
    FILGPU_LIB=crypto3-fil-proofs_amd/build/var/lib_$v.so timeout -k 10 400 python -u bench.py --no-cpu-baseline \
        --no-device-resident --steps ${STEPS:-6} --warmup 1 --msm-reps 2 --tree-log-nodes 0 --sdr-log-labels 0 \
        --config4-log-rows 0 --stacked-log-nodes 0 --uniform-steps 3 --post-reps ${POST_REPS:-1} --winning-reps 10 \
        ${BENCH_ARGS:-} > gpurun_out/ab5/b_${v}_$rep.json 2> gpurun_out/ab5/b_${v}_$rep.err || {
      echo "$v bench FAILED: $(tail -3 gpurun_out/ab5/b_${v}_$rep.err)"; exit 1; }
    echo "$v#$rep: $(python3 -c "
import json; b = json.load(open('gpurun_out/ab5/b_${v}_$rep.json')); t = b['timers_ms']; s = b['steps']
u = b.get('uniform_witness') or {}; w = b.get('winning_post_32gib') or {}; p = b.get('window_post_32gib') or {}
print(round(b['value'] / 1e6, 2), 'Mc/s', round(b['ms_per_step'], 1), 'ms/proof; accum_g1', round(t['accum_g1'] / s, 1),
      'accum_g2', round(t['accum_g2'] / s, 1), 'msm_g1', round(t['msm_g1'] / s, 1), 'ntt', round(t['ntt'] / s, 1),
      'sort', round(t['sort'] / s, 1), '| G1 MSM', round(b['msm_g1_mpoints_per_s'], 1), 'Mpts/s; uniform',
      u.get('ms_per_proof'), 'ms; winning', w.get('latency_ms_median'), 'ms; window', p.get('ms_per_partition_rank0'),
      'ms; micro', (b.get('config2_micro') or {}).get('msm_g1_2e20_ms'), '; verified', b['verified'])")"
  done
done
