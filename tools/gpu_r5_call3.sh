#!/bin/bash
# round 5, third GPU call: kernel timeline of the standalone 2^20 G1 MSM and of the Winning-PoSt leg (the
# small-MSM latency work)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/msm20
timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/msm20/trace -o run -- \
    python3 tools/msm_bench.py --log-rows 20 --reps 20 > gpurun_out/msm20/out.txt 2>&1 || exit 1
cat gpurun_out/msm20/out.txt | tail -2
python3 tools/msm_timeline.py gpurun_out/msm20/trace/run_results.db --reps 10 > gpurun_out/msm20/timeline.md
head -40 gpurun_out/msm20/timeline.md
timeout -k 10 200 python3 tools/msm_bench.py --log-rows 20 --reps 50 || exit 1
bash tools/winning_prof2.sh win6 > /dev/null 2>&1 || exit 1
head -30 gpurun_out/win6/timeline.md
