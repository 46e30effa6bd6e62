# round-4: parity after the small-MSM segment change, then Winning-PoSt A/B against the previous first-level target
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/seg2
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_groth16.py tests/test_gpu_kernels.py \
    > gpurun_out/seg2/tests.log 2>&1 || { tail -30 gpurun_out/seg2/tests.log; exit 1; }
tail -1 gpurun_out/seg2/tests.log
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_post.py \
    -k "winning or small" > gpurun_out/seg2/post.log 2>&1 || { tail -30 gpurun_out/seg2/post.log; exit 1; }
tail -1 gpurun_out/seg2/post.log
B="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 30"
for r in 1 2; do for sa in 0 19; do
    f=gpurun_out/seg2/a${sa}_$r
    if [ "$sa" = 0 ]; then timeout -k 10 180 $B > $f.json 2> $f.err || exit 1
    else MI_MSM_SEGA_LOG=$sa timeout -k 10 180 $B > $f.json 2> $f.err || exit 1; fi
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); w=d['winning_post_32gib']; print('sega=$sa', round(w['latency_ms_median'],2), round(w['latency_ms_min'],2), w['verified'])"
done; done
