#!/bin/bash
# Two-rank rehearsal of bench.py's distributed path on a one-GPU box: both ranks on device 0, gloo for the
# collectives (RCCL refuses two ranks on one device).  Exercises the barrier / max-over-ranks timing, the
# round-robin partition sharding and the multiproof gather exactly as the driver's N-GPU runs do.
# The weak run also exercises the config-5 leg (10 Window-PoSt partitions round-robin, GPU witness + proof)
# with C5 sectors per partition instead of 2349, C5P partitions (default 3: partitions 0 and 1 whole, partition 2
# split over both ranks in latency mode by the balanced schedule).
#   bash tools/dist_rehearsal.sh [log_rows] [config5_sectors] [config5_partitions]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp MI_BENCH_BACKEND=gloo MI_BENCH_SHARED_DEVICE=1
LR=${1:-22}
C5=${2:-64}
C5P=${3:-3}
mkdir -p gpurun_out/dist
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --log-rows "$LR" --no-cpu-baseline \
    --tree-log-nodes 0 --sdr-log-labels 0 --post-sectors "$C5" --post-partitions "$C5P" > gpurun_out/dist/weak.json 2> gpurun_out/dist/weak.err && echo "weak ok: $(cat gpurun_out/dist/weak.json)" &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --gpus 2 --steps 2 --warmup 1 --log-rows "$LR" --partitions 5 --no-cpu-baseline \
    --tree-log-nodes 0 --sdr-log-labels 0 --post-sectors 0 > gpurun_out/dist/p5.json 2> gpurun_out/dist/p5.err && echo "partitions ok: $(cat gpurun_out/dist/p5.json)"
