#!/bin/bash
# A/B NTT builds on one box: build/var/lib_<v>.so first run the NTT kernel tests (correctness), then
# tools/ntt_bench.py alternately (same box, same run).
set -e
cd "$GRAFT_REPO_ROOT"
V=${1:-"a b"}
mkdir -p gpurun_out/var
for v in $V; do
  FILGPU_LIB=crypto3-fil-proofs_amd/build/var/lib_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -k ntt -x -q --timeout 120 --timeout-method thread > gpurun_out/var/nt_$v.log 2>&1
  echo "$v tests: $(tail -1 gpurun_out/var/nt_$v.log)"
done
for rep in 1 2 3; do
  for v in $V; do
    FILGPU_LIB=crypto3-fil-proofs_amd/build/var/lib_$v.so timeout -k 10 120 python -u tools/ntt_bench.py --log 26 --reps 5 > gpurun_out/var/n_${v}_$rep.log 2>&1
    echo "$v#$rep: $(grep -o 'passes [0-9.]*' gpurun_out/var/n_${v}_$rep.log | tr '\n' ' ')"
  done
done
