#!/bin/bash
# round 5, first GPU call: maddloop old vs new field (same box), then the GPU parity suites on the new build
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5c1
timeout -k 10 240 crypto3-fil-proofs_amd/build/var/maddloop_old 64 2.0 > gpurun_out/r5c1/madd_old.jsonl 2>&1 || exit 1
timeout -k 10 240 crypto3-fil-proofs_amd/build/var/maddloop_new 64 2.0 > gpurun_out/r5c1/madd_new.jsonl 2>&1 || exit 1
echo "maddloop done"
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_groth16.py tests/test_gpu_cpp.py -x -v \
    --timeout 300 --timeout-method thread > gpurun_out/r5c1/tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5c1/tests.log
exit $rc
