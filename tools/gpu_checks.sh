#!/bin/bash
# GPU checks of round 5, one mode per gpurun call (each step under its own time limit; stops at the first failure):
#   parity    the MSM / proof / PoSt parity tests (window tables, plans, every lane layout; not the 64 GiB test)
#   winning   Winning-PoSt latency leg of bench.py, two runs of 20 calls
#   msm20     the 2^20 G1 MSM over a window table (c = 20) and plain (tools/msm_bench.py)
#   trace     Winning-PoSt breakdown: rocprofv3 kernel + HIP runtime traces (databases in /tmp), timelines to $O
#   suite     the whole GPU suite and smoke(), as the driver runs them
#   post64    the 64 GiB Window-PoSt partition test with its record lines
#   witness   the stacked / PoSt witness and Poseidon parity tests
#   bench     the default bench line (python3 bench.py) into $O/bench.json
#   c3ab      the config-3 main leg, default and with each switch of C3AB="name=value ..." (alternated twice)
#   wpab      the Window-PoSt leg, default and with each switch of WPAB="name=value ..." (--tune A/B)
# usage: /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/gpu_checks.sh parity winning
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/checks
mkdir -p $O
W="python3 bench.py --steps 1 --warmup 0 --log-rows 12 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0"
for mode in "$@"; do
  case $mode in
    parity)
      timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
          tests/test_gpu_groth16.py tests/test_gpu_post.py -k "not 64gib" > $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
      tail -1 $O/parity.log ;;
    winning)
      for v in a b; do
        timeout -k 10 300 $W --winning-reps 20 > $O/win_$v.json 2> $O/win_$v.err || exit 1
        python3 -c "import json; w = json.load(open('$O/win_$v.json'))['winning_post_32gib']; print('winning', round(w['latency_ms_median'], 2), round(w['latency_ms_min'], 2), w['verified'])"
      done ;;
    msm20)
      timeout -k 10 200 python3 tools/msm_bench.py --log-rows 20 --reps 50 --table 20 2>&1 | grep "G1 MSM" || exit 1
      timeout -k 10 200 python3 tools/msm_bench.py --log-rows 20 --reps 50 --tune msm_wt=0 2>&1 | grep "G1 MSM" || exit 1 ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d /tmp/wintrace -o run -- \
          $W --winning-reps 10 > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
      python3 tools/winning_timeline.py /tmp/wintrace/run_results.db --md > $O/timeline.md
      python3 tools/call_timeline.py /tmp/wintrace/run_results.db --kernels --min-ms 0.2 > $O/call.txt
      cat $O/timeline.md; grep "^stream\|gaps\|host tid" $O/call.txt ;;
    suite)
      timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
      tail -1 $O/gpu_tests.log
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
      tail -1 $O/smoke.log ;;
    witness)
      timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stacked.py \
          tests/test_gpu_post.py tests/test_gpu_poseidon.py -k "not 64gib" > $O/witness.log 2>&1 || { tail -20 $O/witness.log; exit 1; }
      tail -1 $O/witness.log ;;
    bench)
      timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
      tail -c 400 $O/bench.json ;;
    wpab)  # the 32 GiB Window-PoSt leg (two lanes, as the driver bench runs it), default and with each WPAB switch
      for v in default ${WPAB:-}; do
        T=(); [ "$v" = default ] || for kv in ${v//,/ }; do T+=(--tune "$kv"); done
        timeout -k 10 300 $W --post-sectors 2349 --post-reps 2 --post-share-groups "" --winning-log-nodes 0 "${T[@]}" > $O/wp_$v.json 2> $O/wp_$v.err || { tail -5 $O/wp_$v.err; exit 1; }
        python3 -c "import json; w = json.load(open('$O/wp_$v.json'))['window_post_32gib']; print('window-post $v', round(w['ms_per_partition_rank0'], 1), w['verified'])"
      done ;;
    c3ab)  # config-3 main leg (5 timed proofs), default and each C3AB switch, alternated twice (same box)
      for rep in 1 2; do
        for v in default ${C3AB:-}; do
          T=(); [ "$v" = default ] || for kv in ${v//,/ }; do T+=(--tune "$kv"); done
          timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --msm-reps 1 --no-cpu-baseline --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --config4-log-rows 0 --stacked-log-nodes 0 --post-sectors 0 --uniform-steps 0 --winning-log-nodes 0 "${T[@]}" > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
          python3 -c "import json; d = json.load(open('$O/c3_$v.json')); print('config3 $v', round(d['ms_per_step'], 2), round(d['value'] / 1e6, 2), 'Mc/s')"
        done
      done ;;
    post64)
      timeout -k 10 900 python3 -u -m pytest -x -q -s --timeout 800 --timeout-method thread tests/test_gpu_post.py -k 64gib > $O/post64.log 2>&1 || exit 1
      grep "window-post-64\|passed" $O/post64.log ;;
    *) echo "unknown mode $mode"; exit 2 ;;
  esac
done
