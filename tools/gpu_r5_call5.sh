#!/bin/bash
# round 5, fifth GPU call: parity after the one-readback plan refactor, then kernel timelines of the 2^20 MSM over
# window tables at c = 16 / 18 / 20 and without a table
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c5
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_groth16.py > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for t in 16 18 20 none; do
  if [ $t = none ]; then A="MI_MSM_WT=0"; T=0; else A="MI_MSM_WT=1"; T=$t; fi
  env $A timeout -k 10 240 rocprofv3 --kernel-trace -d $O/tr_$t -o run -- python3 tools/msm_bench.py --log-rows 20 --reps 20 --table $T > $O/msm_$t.txt 2>&1 || exit 1
  tail -1 $O/msm_$t.txt
  python3 tools/msm_timeline.py $O/tr_$t/run_results.db --reps 10 > $O/timeline_$t.md
  head -24 $O/timeline_$t.md
done
