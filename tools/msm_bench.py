#!/usr/bin/env python3
"""Standalone G1 MSM timing over the resident h-query points of a generated 2^L proving key
(random dense scalars, device-resident), with the library's phase timers (sort / accumulation /
whole MSM).  Used to tune MSM phases in isolation from the two-lane prove.

    python tools/msm_bench.py --log-rows 26 --reps 3
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "crypto3-fil-proofs_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-rows", type=int, default=26)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--query", type=int, default=0, help="0 h, 1 l, 2 a, 3 b_g1, 4 b_g2")
    ap.add_argument("--table", type=int, default=-1, help="window-table bits (0 = library choice; -1 none)")
    ap.add_argument("--n", type=int, default=0, help="points (default: the whole query)")
    ap.add_argument("--tune", action="append", default=[], metavar="NAME=VALUE", help="library A/B switch (mi_tune_set)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import fil_groth16 as fg

    for kv in a.tune:
        k, _, v = kv.partition("=")
        fg.tune_set(k, int(v))
    from fil_groth16 import synth
    from bench import TOXIC_SEED, splitmix_frs

    ctx = fg.Context(0)
    sc = synth.SynthCircuit(a.log_rows, 4, 1)
    circ = sc.load(ctx)
    pk = fg.generate_random_parameters(ctx, circ, splitmix_frs(TOXIC_SEED, 5))
    pts = pk.points(a.query)
    n = a.n or pts.n
    if a.table >= 0:
        t = time.perf_counter()
        pts.precompute(a.table, n)
        ctx.synchronize()
        print(f"table {pts.table_info()} built in {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
    rng = np.random.default_rng(7)
    sw = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    sw[:, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)
    s_dev = torch.from_numpy(sw.view(np.uint8).reshape(-1)).to("cuda")
    pts.msm_dev(s_dev.data_ptr(), n)
    ctx.synchronize()
    ctx.reset_stats()
    t = time.perf_counter()
    for _ in range(a.reps):
        pts.msm_dev(s_dev.data_ptr(), n)
    ctx.synchronize()
    dt = (time.perf_counter() - t) / a.reps * 1e3
    st = ctx.stats()
    grp = "g2" if a.query == 4 else "g1"
    per = {k: round(st[k]["ms"] / a.reps, 2) for k in ("sort", "accum_" + grp, "msm_" + grp)}
    print(f"{grp.upper()} MSM query={a.query} table={pts.table_info()['window_bits']} n={n}: {dt:.1f} ms wall ({n / dt / 1e3:.1f} Mpts/s); per MSM {per}", flush=True)


if __name__ == "__main__":
    main()
