# round-4: small-proof lanes (B, L, A on lanes of their own) -- parity tests, then Winning-PoSt A/B against two lanes
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/lanes
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_groth16.py \
    -k "lane_layouts or golden or random_vs_oracle or share or trapdoor or split_msm or batch" \
    > gpurun_out/lanes/tests.log 2>&1 || { tail -30 gpurun_out/lanes/tests.log; exit 1; }
tail -3 gpurun_out/lanes/tests.log
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_post.py \
    -k "winning" > gpurun_out/lanes/post.log 2>&1 || { tail -30 gpurun_out/lanes/post.log; exit 1; }
tail -3 gpurun_out/lanes/post.log
B="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 20"
for r in 1 2; do for v in 21:0 0:0 21:1 21:2; do
    w=${v%:*}; b1=${v#*:}; f=gpurun_out/lanes/w${w}_b${b1}_$r
    MI_PROVE_WIDE_LOG=$w MI_PROVE_B1_LANE=$b1 timeout -k 10 180 $B > $f.json 2> $f.err || exit 1
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1])['winning_post_32gib']; print('wide_log=$w b1_lane=$b1', round(d['latency_ms_median'],2), round(d['latency_ms_min'],2), d['verified'])"
done; done
