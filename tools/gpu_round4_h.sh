#!/bin/bash
# round-4: phase-B Poseidon on lanes -- every witness test against the oracle, the smoke, then the stacked /
# Window-PoSt / Winning-PoSt legs
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_stacked.py tests/test_gpu_post.py tests/test_gpu_memory.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests8.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r04_gpu_tests8.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke2.log 2>&1 || exit 1
tail -1 gpurun_out/r04_smoke2.log
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --log-rows 20 --no-cpu-baseline --no-device-resident --config4-log-rows 0 --tree-log-nodes 0 --sdr-log-labels 0 --uniform-steps 0 --winning-reps 20 > gpurun_out/r04_bench_legs3.json 2> gpurun_out/r04_bench_legs3.err
echo "bench rc=$?"
python3 - <<PY
import json
d = json.loads(open("gpurun_out/r04_bench_legs3.json").read().strip().splitlines()[-1])
w, s, p = d["winning_post_32gib"], d["stacked_porep_32gib"], d["window_post_32gib"]
print("winning", round(w["latency_ms_median"], 2), w["device_ms_per_proof"])
print("stacked", round(s["witness_ms"], 2), s["witness_phases_ms_per_partition"], round(s["witness_plus_prove_ms"], 1), s["verified"])
print("window", round(p["ms_per_partition_rank0"], 1), round(p["witness_ms_per_partition_rank0"], 2), p["verified"])
PY
