#!/bin/bash
# GPU tests + one bench line on the box (each GPU step under its own time limit, chained with &&).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${T_TESTS:-800} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
    > gpurun_out/tests.log 2>&1 && echo "tests ok" &&
timeout -k 10 ${T_BENCH:-300} python -u bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-2} ${BENCH_ARGS:-} \
    > gpurun_out/bench.json 2> gpurun_out/bench.err && echo "bench ok"
