"""SDR labelling-witness throughput alone (bench.py's sdr_leg): one JSON line.  Used for
the rocprofv3 kernel trace of k_sdr_labels_gather without the Groth16 run around it.
   python tools/sdr_bench.py [--log-labels 24] [--no-cpu-baseline]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-labels", type=int, default=24)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()
    import torch

    import bench
    import fil_groth16 as fg

    args = argparse.Namespace(sdr_log_labels=a.log_labels, no_cpu_baseline=a.no_cpu_baseline)
    ctx = fg.Context(0)
    dev = torch.device("cuda:0")
    res = bench.sdr_leg(args, fg, ctx, dev, 1)
    # the per-entry form (k_sdr_labels): 14 parents per label given contiguously, the same hash work with
    # streaming reads instead of random gathers -- separates the VALU bound from the gather traffic
    import time

    n = 1 << a.log_labels
    par = torch.randint(0, 256, (n * 14 * 32,), dtype=torch.uint8, device=dev)
    lay = torch.randint(2, 12, (n,), dtype=torch.int32, device=dev)
    nod = torch.randint(1, 1 << 30, (n,), dtype=torch.int64, device=dev)
    out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    run = lambda: fg.sdr.create_labels_dev(ctx, bytes(32), n, lay.data_ptr(), nod.data_ptr(), par.data_ptr(), 14,
                                           out.data_ptr())
    run()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        run()
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / 5
    res["per_entry_form"] = {"kernel": "k_sdr_labels", "labels_per_s": n / dt, "ms_per_batch": dt * 1e3,
                             "valu_frac": n * 20 * bench.SHA256_OPS_PER_COMPRESSION / dt / bench.VALU_LANE_OPS}
    # tree D (binary SHA-256 tree over the data, comm_d): 2^log_labels leaves, 2 compressions per node
    leaves = torch.randint(0, 256, (n * 32,), dtype=torch.uint8, device=dev)
    tree = torch.empty((n - 1) * 32, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    fg.sdr.build_tree_d_dev(ctx, leaves.data_ptr(), n, tree.data_ptr())
    t0 = time.perf_counter()
    for _ in range(5):
        fg.sdr.build_tree_d_dev(ctx, leaves.data_ptr(), n, tree.data_ptr())
    dt = (time.perf_counter() - t0) / 5
    res["tree_d"] = {"kernel": "k_sha256_pairs (one launch per level)", "leaves": n, "ms_per_tree": dt * 1e3,
                     "leaves_per_s": n / dt, "GB_per_s_of_data": n * 32 / dt / 1e9,
                     "valu_frac": (n - 1) * 2 * bench.SHA256_OPS_PER_COMPRESSION / dt / bench.VALU_LANE_OPS}
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
