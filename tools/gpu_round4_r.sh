# round-4: Winning-PoSt latency vs the bucket reduction's segment sizes (MI_MSM_SEGB_LOG, MI_MSM_SEGA_LOG)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/seg
B="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-reps 30"
for v in 0:0 10:0 12:0 9:0 0:17 0:16 11:17 0:0; do
    sb=${v%:*}; sa=${v#*:}; f=gpurun_out/seg/b${sb}_a${sa}
    env_args=""
    [ "$sb" != 0 ] && env_args="$env_args MI_MSM_SEGB_LOG=$sb"
    [ "$sa" != 0 ] && env_args="$env_args MI_MSM_SEGA_LOG=$sa"
    env $env_args timeout -k 10 180 $B > $f.json 2> $f.err || exit 1
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); w=d['winning_post_32gib']; print('segb=$sb sega=$sa', round(w['latency_ms_median'],2), round(w['latency_ms_min'],2), w['verified'], 'msm2e20', round(d.get('config2_micro',{}).get('msm_g1_2e20_ms',0),3))"
done
