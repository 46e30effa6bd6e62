#!/bin/bash
# round-4 GPU check: the full -m gpu suite, the batch-affine microbenchmark, then the default bench line
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests3.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/r04_gpu_tests3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd crypto3-fil-proofs_amd/microbench && timeout -k 10 240 ./maddloop 64 2.0 ba > ../../gpurun_out/r04_maddloop_ba.jsonl 2>&1
rc=$?; cd ../..
echo "maddloop rc=$rc"; cat gpurun_out/r04_maddloop_ba.jsonl
