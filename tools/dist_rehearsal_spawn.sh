#!/bin/bash
# The driver's multi-GPU command form, `bench.py --gpus N` with no launcher, rehearsed on a one-GPU box: every rank
# on device 0 (MI_BENCH_SHARED_DEVICE=1), gloo for the collectives (RCCL refuses two ranks on one device), small
# Window-PoSt partitions.  N = 4: 10 partitions -> 8 whole + 2 tail partitions over groups of 2;
# N = 8: 8 whole + 2 tail partitions over groups of 4 (the config-5 schedule).
cd "$GRAFT_REPO_ROOT" || exit 1
export MI_BENCH_BACKEND=gloo MI_BENCH_SHARED_DEVICE=1
mkdir -p gpurun_out/spawn
for n in ${RANKS:-4 8}; do
    timeout -k 10 400 python3 bench.py --gpus $n --steps 2 --warmup 1 --log-rows 16 --msm-reps 1 --no-cpu-baseline \
        --no-device-resident --tree-log-nodes 0 --sdr-log-labels 0 --post-sectors 16 --post-log-nodes 12 \
        --post-partitions 10 > gpurun_out/spawn/n$n.json 2> gpurun_out/spawn/n$n.err || { echo "n=$n failed"; tail -20 gpurun_out/spawn/n$n.err; exit 1; }
    python3 - <<PY
import json
d = json.loads(open("gpurun_out/spawn/n$n.json").read().strip().splitlines()[-1])
c = d["config5"]
print("n_gpus", d["n_gpus"], "main verified", d["verified"], d["verified_proofs"], "| config5:", {k: c.get(k) for k in
      ("n_gpus", "partitions", "verified", "verified_proofs", "schedule", "latency_mode", "per_rank_partitions",
       "split_partitions", "makespan_s", "latency_mode_calibration_ms", "error")})
PY
done
