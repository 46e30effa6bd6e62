#!/bin/bash
# round 5, second GPU call: maddloop old vs new field (same box), parity gate on the new build, then the prove A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5c2
timeout -k 10 240 crypto3-fil-proofs_amd/build/var/maddloop_old 64 2.0 > gpurun_out/r5c2/madd_old.jsonl 2>&1 || exit 1
timeout -k 10 240 crypto3-fil-proofs_amd/build/var/maddloop_new 64 2.0 > gpurun_out/r5c2/madd_new.jsonl 2>&1 || exit 1
grep -h '"gather128"\|"g2_gather224"' gpurun_out/r5c2/madd_old.jsonl gpurun_out/r5c2/madd_new.jsonl | cut -c1-120
TEST_VARIANTS=new bash tools/gpu_r5_ab.sh "old new" 2
