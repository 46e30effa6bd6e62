# round-4: Winning-PoSt latency with more hardware queues per process (lanes sharing a queue serialise)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/hwq
B="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 30"
for r in 1 2; do for v in 4:21 8:21 4:0 8:0; do
    q=${v%:*}; w=${v#*:}; f=gpurun_out/hwq/q${q}_w${w}_$r
    GPU_MAX_HW_QUEUES=$q MI_PROVE_WIDE_LOG=$w timeout -k 10 180 $B > $f.json 2> $f.err || exit 1
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); w=d['winning_post_32gib']; print('hwq=$q wide_log=$w', round(w['latency_ms_median'],2), round(w['latency_ms_min'],2), w['verified'])"
done; done
