#!/bin/bash
# A/B NTT timing: build/var/lib_<v>.so alternately through tools/ntt_bench.py (same box, same run).
set -e
cd "$GRAFT_REPO_ROOT"
V=${1:-"a b"}
mkdir -p gpurun_out/var
for rep in 1 2 3; do
  for v in $V; do
    FILGPU_LIB=crypto3-fil-proofs_amd/build/var/lib_$v.so timeout -k 10 120 python -u tools/ntt_bench.py --log 26 --reps 5 > gpurun_out/var/n_${v}_$rep.log 2>&1
    echo "$v#$rep: $(grep log gpurun_out/var/n_${v}_$rep.log | sed 's/ms\/transform wall, passes/|/' | awk '{print $NF}' | tr '\n' ' ')"
  done
done
