mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_memory.py tests/test_gpu_post.py tests/test_gpu_poseidon.py tests/test_gpu_scale.py tests/test_gpu_sdr.py tests/test_gpu_stacked.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests2.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/r04_gpu_tests2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd crypto3-fil-proofs_amd/microbench && timeout -k 10 240 ./maddloop 64 2.0 ba > ../../gpurun_out/r04_maddloop_ba.jsonl 2>&1
echo "maddloop rc=$?"; cat ../../gpurun_out/r04_maddloop_ba.jsonl
