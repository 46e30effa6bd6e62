# round-4: Winning-PoSt latency across lane layouts and second-level reduction segments
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/lanes3
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_groth16.py \
    > gpurun_out/lanes3/tests.log 2>&1 || { tail -30 gpurun_out/lanes3/tests.log; exit 1; }
tail -1 gpurun_out/lanes3/tests.log
B="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 30"
for r in 1 2; do for v in 21:0:0 0:0:0 21:2:0 21:0:13 0:0:13; do
    IFS=: read w b1 sb <<< "$v"; f=gpurun_out/lanes3/w${w}_b${b1}_s${sb}_$r
    if [ "$sb" = 0 ]; then MI_PROVE_WIDE_LOG=$w MI_PROVE_B1_LANE=$b1 timeout -k 10 180 $B > $f.json 2> $f.err || exit 1
    else MI_MSM_SEGB_LOG=$sb MI_PROVE_WIDE_LOG=$w MI_PROVE_B1_LANE=$b1 timeout -k 10 180 $B > $f.json 2> $f.err || exit 1; fi
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); w=d['winning_post_32gib']; print('wide_log=$w b1_lane=$b1 segb=$sb', round(w['latency_ms_median'],2), round(w['latency_ms_min'],2), w['verified'], 'msm2e20', round(d['config2_micro']['msm_g1_2e20_ms'],3))"
done; done
