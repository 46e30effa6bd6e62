#!/usr/bin/env python3
"""Time device-resident NTTs (mi_ntt_fr_dev) at 2^L: per-transform wall time and the library's
NTT-pass timer.  Used to tune the pass kernel.

    python tools/ntt_bench.py --log 26 --reps 5
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "crypto3-fil-proofs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log", type=int, default=26)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import fil_groth16 as fg

    ctx = fg.Context(0)
    n = 1 << a.log
    x = torch.randint(0, 2**31 - 1, (n, 8), dtype=torch.int32, device="cuda")
    x[:, 7] &= 0x0FFFFFFF  # < r
    ptr = x.data_ptr()
    for kind in [(False, False), (True, False), (False, True)]:
        ctx.ntt_dev(ptr, a.log, *kind)
        torch.cuda.synchronize()
        ctx.reset_stats()
        t = time.perf_counter()
        for _ in range(a.reps):
            ctx.ntt_dev(ptr, a.log, *kind)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.reps * 1e3
        st = ctx.stats()
        print(f"log {a.log} inverse={kind[0]} coset={kind[1]}: {dt:.2f} ms/transform wall, "
              f"passes {st['ntt']['ms'] / max(1, st['ntt']['launches']):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
