#!/bin/bash
# round 5, fourteenth GPU call: same-box A/B of the G2 reduction kernels with and without the two-wave register cap
# (G2 parity on the uncapped build first)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TEST_VARIANTS=g2nc TESTS="tests/test_gpu_kernels.py tests/test_gpu_scale.py" TESTK="g2 or G2" STEPS=6 bash tools/gpu_r5_ab.sh "cur g2nc" 2
