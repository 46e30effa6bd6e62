#!/usr/bin/env python3
"""Tree C / tree R-last / Poseidon throughput on one GPU, device-resident inputs.

Workload: one sub-tree of a 32 GiB sector at 2^log_nodes nodes (2^27 for 32 GiB's 8 sub-trees; default
2^24 so a run takes seconds): 11 layers of labels -> column hashes (Poseidon, arity 11) -> arity-8 tree
(tree C); last-layer labels + data -> replica -> arity-8 tree with rows_to_discard = 2 (tree R-last).
Prints one JSON line: columns/s, leaves/s, per-arity hashes/s, and the VALU roofline of k_poseidon
(v_mad_u64_u32 issue: one Fr product = 162 MADs over 9 x 29-bit limbs, a square 126 (symmetric
products); an MDS row of K <= 6 terms = 81 K + 81 MADs).
    python tools/tree_bench.py [--log-nodes 24] [--reps 3]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "crypto3-fil-proofs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

MAD_RATE = 1024 * 64 / 4 * 2.4e9  # lane-MADs/s: 1024 SIMDs, wave64, 4 cycles per v_mad_u64_u32, 2.4 GHz
ROUNDS = {2: 55, 4: 56, 8: 57, 11: 57}


def mads_per_hash(arity):
    t, rp, rf = arity + 1, ROUNDS[arity], 8
    mul = 162
    sbox = 2 * 126 + mul  # x^2, x^4 as symmetric squares (fr29_sqr), x^5

    def row(k):  # t-term row in chunks of <= 6 products per reduction
        if k <= 6:
            return 81 * k + 81
        a = (k + 1) // 2
        return row(a) + row(k - a)

    full = rf * (t * sbox + t * row(t))
    sparse = (rp - 1) * (sbox + row(t) + (t - 1) * mul)
    last = sbox + t * row(t)
    io = (t - 1) * mul + mul
    return full + sparse + last + io


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-nodes", type=int, default=24)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--layers", type=int, default=11)
    a = ap.parse_args()
    import numpy as np
    import torch
    import fil_groth16 as fg
    from fil_groth16._lib import check, lib

    ctx = fg.Context(0)
    n = 1 << a.log_nodes
    L = a.layers
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    # canonical Fr labels: 4 random u64 words, top word masked below r's top word
    labels = torch.randint(0, 2 ** 62, (L * n, 4), dtype=torch.int64, device="cuda", generator=g)
    labels[:, 3] &= 0x0FFFFFFFFFFFFFFF
    data = torch.randint(0, 2 ** 62, (n, 4), dtype=torch.int64, device="cuda", generator=g)
    data[:, 3] &= 0x0FFFFFFFFFFFFFFF
    base = torch.empty((n, 4), dtype=torch.int64, device="cuda")
    tsz_c = fg.tree.get_merkle_tree_cache_size(n, 8, 0)
    tree_c = torch.empty((tsz_c, 4), dtype=torch.int64, device="cuda")
    disc = fg.tree.default_rows_to_discard(n, 8)
    tsz_r = fg.tree.get_merkle_tree_cache_size(n, 8, disc)
    tree_r = torch.empty((max(tsz_r, 1), 4), dtype=torch.int64, device="cuda")
    builder = fg.tree.ColumnTreeBuilder(ctx, L, 8)
    vp = ctypes.c_void_p

    def run_c():
        builder.add_final_columns_dev(labels.data_ptr(), n, base.data_ptr(), tree_c.data_ptr())

    def run_r():
        d = data.clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fg.tree.generate_tree_r_last_dev(ctx, n, labels[(L - 1) * n:].data_ptr(), d.data_ptr(), tree_r.data_ptr(), 8,
                                         disc)
        ctx.synchronize()
        return time.perf_counter() - t0

    run_c()
    ctx.synchronize()
    ctx.reset_stats()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        run_c()
    ctx.synchronize()
    tc = (time.perf_counter() - t0) / a.reps
    st = ctx.stats()["poseidon"]
    run_r()
    tr = min(run_r() for _ in range(a.reps))
    # per-arity hash rates (n / 8 hashes each, device-resident preimages)
    rates = {}
    for ar in (2, 8, 11):
        cnt = min(n, (L * n) // ar)
        out = torch.empty((cnt, 4), dtype=torch.int64, device="cuda")
        fg.tree.poseidon_hash_dev(ctx, ar, labels.data_ptr(), cnt, out.data_ptr())
        ctx.synchronize()
        ctx.reset_stats()
        for _ in range(a.reps):
            fg.tree.poseidon_hash_dev(ctx, ar, labels.data_ptr(), cnt, out.data_ptr())
        ctx.synchronize()
        s = ctx.stats()["poseidon"]
        rates[str(ar)] = {"hashes_per_s": s["units"] / (s["ms"] * 1e-3), "avg_launch_ms": s["ms"] / s["launches"],
                          "hashes_per_launch": cnt}
        del out
    r11 = rates[str(L)] if str(L) in rates else None
    mads = mads_per_hash(L)
    peak_h = MAD_RATE / mads
    col_kernel_ms = r11["avg_launch_ms"] if r11 else None
    out = {
        "metric": "tree C columns/s (Poseidon arity-11 column hashes + arity-8 tree), device-resident labels",
        "workload": f"one sub-tree of 2^{a.log_nodes} nodes x {L} layers (32 GiB sector = 8 sub-trees of 2^27)",
        "tree_c_s": tc, "tree_c_columns_per_s": n / tc,
        "tree_r_last_s": tr, "tree_r_last_leaves_per_s": n / tr, "tree_r_last_rows_to_discard": disc,
        "poseidon": rates,
        "valu_roofline": {
            "kernel": f"k_poseidon<{L + 1}>", "bound": "valu (v_mad_u64_u32 issue)",
            "mads_per_hash": mads, "achieved_hashes_per_s": r11["hashes_per_s"] if r11 else None,
            "peak_hashes_per_s": peak_h, "frac": (r11["hashes_per_s"] / peak_h) if r11 else None,
        },
        "hbm_roofline": {
            "kernel": f"k_poseidon<{L + 1}>", "bound": "hbm", "algorithmic_bytes_per_hash": 32 * L + 32,
            "achieved_GBps": (r11["hashes_per_s"] * (32 * L + 32) / 1e9) if r11 else None, "peak_GBps": 8000.0,
        },
        "tree_c_launch_stats": st,
        "projected_32GiB_sector_tree_c_s": tc * (2 ** 27 / n) * 8,
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
