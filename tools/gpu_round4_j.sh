#!/bin/bash
# round-4 final: every -m gpu test, the smoke, the default bench line (the driver's command), the one-lane trace
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests_final.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r04_gpu_tests_final.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke_final.log 2>&1 || exit 1
tail -1 gpurun_out/r04_smoke_final.log
