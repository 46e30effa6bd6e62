#!/bin/bash
# round-4: lanes only for small Poseidon launches -- witness tests, legs, then the Window-PoSt trace
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_stacked.py tests/test_gpu_post.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests9.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r04_gpu_tests9.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --log-rows 20 --no-cpu-baseline --no-device-resident --config4-log-rows 0 --tree-log-nodes 0 --sdr-log-labels 0 --uniform-steps 0 --winning-reps 20 > gpurun_out/r04_bench_legs4.json 2> gpurun_out/r04_bench_legs4.err
echo "bench rc=$?"
python3 - <<PY
import json
d = json.loads(open("gpurun_out/r04_bench_legs4.json").read().strip().splitlines()[-1])
w, s, p = d["winning_post_32gib"], d["stacked_porep_32gib"], d["window_post_32gib"]
print("winning", round(w["latency_ms_median"], 2), w["device_ms_per_proof"])
print("stacked", round(s["witness_ms"], 2), s["witness_phases_ms_per_partition"], round(s["witness_plus_prove_ms"], 1), s["verified"])
print("window", round(p["ms_per_partition_rank0"], 1), round(p["witness_ms_per_partition_rank0"], 2), p["verified"], {g: v["slowest_ms"] for g, v in p["latency_mode_shares"].items()})
PY
bash tools/window_prof.sh winpost
