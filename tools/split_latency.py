"""Single-proof latency mode on one GPU: time every rank's share of a 2^log-rows proof for world
sizes W, one rank after another, and check that the assembled shares give the one-GPU proof bytes.

On a W-GPU node the ranks run concurrently, so the proof latency is max over ranks of the share time
plus the 576-byte all-gather and the host assembly; this script reports that projection next to the
measured one-GPU prove.  Usage: python tools/split_latency.py [--log-rows 26] [--worlds 2 4 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "crypto3-fil-proofs_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-rows", type=int, default=26)
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch

    import fil_groth16 as fg
    from bench import TOXIC_SEED, splitmix_frs
    from fil_groth16 import synth

    ctx = fg.Context(0)
    sc = synth.SynthCircuit(args.log_rows, 4, 1)
    circ = sc.load(ctx)
    pk = fg.generate_random_parameters(ctx, circ, splitmix_frs(TOXIC_SEED, 5))
    z = torch.from_numpy(sc.z_array().copy()).cuda()
    torch.cuda.synchronize()
    vk, _ = pk.verifying_key()
    r, s = splitmix_frs(77, 2)

    def timed(fn):
        best, out = None, None
        for _ in range(args.reps):
            t0 = time.perf_counter()
            out = fn()
            ctx.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return best, out

    fg.prove(ctx, pk, circ, z.data_ptr(), r, s)  # warm-up
    t_one, proof = timed(lambda: fg.prove(ctx, pk, circ, z.data_ptr(), r, s))
    res = {"workload": f"synthetic 2^{args.log_rows}-constraint prove", "n": sc.n, "one_gpu_ms": 1e3 * t_one,
           "split": []}
    print(f"one GPU: {1e3 * t_one:.1f} ms", flush=True)
    for w in args.worlds:
        times, shares = [], []
        for k in range(w):
            t, sh = timed(lambda: fg.prove_share(ctx, pk, circ, z.data_ptr(), k, w))
            times.append(1e3 * t)
            shares.append(sh)
        t0 = time.perf_counter()
        p = fg.assemble(vk, shares, r, s)
        t_asm = 1e3 * (time.perf_counter() - t0)
        ok = p == proof
        res["split"].append({"world": w, "share_ms": times, "assemble_ms": t_asm, "bit_exact": ok,
                             "projected_latency_ms": max(times) + t_asm,
                             "speedup": t_one * 1e3 / (max(times) + t_asm)})
        print(f"W={w}: shares {min(times):.1f}..{max(times):.1f} ms, assemble {t_asm:.1f} ms, "
              f"projected latency {max(times) + t_asm:.1f} ms, bit-exact {ok}", flush=True)
        if not ok:
            raise SystemExit("assembled shares differ from the one-GPU proof")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
