#!/bin/bash
# A/B variant timing on one GPU box: each build/var/lib_<v>.so runs the MSM kernel tests once
# (correctness), then the standalone MSM bench, alternating variants so box-level drift shows up.
#   bash tools/variants.sh "a b c" <query> <log_rows>
set -e
cd "$GRAFT_REPO_ROOT"
V=${1:-"a b"}; Q=${2:-0}; LR=${3:-26}
mkdir -p gpurun_out/var
for v in $V; do
  FILGPU_LIB=crypto3-fil-proofs_amd/build/var/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k msm -x -q --timeout 200 --timeout-method thread > gpurun_out/var/t_$v.log 2>&1
  echo "$v tests: $(tail -1 gpurun_out/var/t_$v.log)"
done
for rep in 1 2; do
  for v in $V; do
    FILGPU_LIB=crypto3-fil-proofs_amd/build/var/lib_$v.so timeout -k 10 200 python -u tools/msm_bench.py --log-rows $LR --reps 3 --query $Q > gpurun_out/var/b_${v}_$rep.log 2>&1
    echo "$v#$rep: $(tail -1 gpurun_out/var/b_${v}_$rep.log)"
  done
done
