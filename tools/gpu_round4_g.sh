#!/bin/bash
# round-4: split-threshold change checked (MSM / proof tests, smoke), Winning-PoSt + 2^20 MSM numbers, then the
# round's rocprofv3 evidence of the headline (kernel trace + FETCH_SIZE + WRITE_SIZE passes)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_groth16.py tests/test_gpu_kernels.py tests/test_gpu_scale.py tests/test_gpu_post.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests7.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r04_gpu_tests7.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r04_smoke.log
SPLIT_SWEEP="def 16 def" bash tools/split_sweep.sh || exit 1
bash tools/prof_round.sh r04 || exit 1
ls gpurun_out/r04_trace gpurun_out/r04_fetch | head
