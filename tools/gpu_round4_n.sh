# round-4: pinned readbacks + blind terms off the critical path -- parity, Winning-PoSt A/B, trace
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/lanes2
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_groth16.py \
    > gpurun_out/lanes2/tests.log 2>&1 || { tail -30 gpurun_out/lanes2/tests.log; exit 1; }
tail -2 gpurun_out/lanes2/tests.log
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_post.py \
    -k "winning or small" > gpurun_out/lanes2/post.log 2>&1 || { tail -30 gpurun_out/lanes2/post.log; exit 1; }
tail -2 gpurun_out/lanes2/post.log
B="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 20"
for r in 1 2; do for w in 21 0; do
    f=gpurun_out/lanes2/w${w}_$r
    MI_PROVE_WIDE_LOG=$w timeout -k 10 180 $B > $f.json 2> $f.err || exit 1
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1])['winning_post_32gib']; print('wide_log=$w', round(d['latency_ms_median'],2), round(d['latency_ms_min'],2), d['verified'])"
done; done
bash tools/winning_prof2.sh win4
