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
    res = bench.sdr_leg(args, fg, ctx, torch.device("cuda:0"), 1)
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
