#!/usr/bin/env python3
"""Device memory at each stage of one 32 GiB partition (build, load, keygen, witness, prove): the working
set behind the split-table decision, and back-to-back proofs for a rocprofv3 lane timeline.
    python tools/post_mem.py [sectors | stacked] [proofs]
sectors (default 2349): a Window-PoSt partition; "stacked": the 32 GiB stacked-PoRep partition."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "crypto3-fil-proofs_amd")
import fil_groth16 as fg  # noqa: E402
from fil_groth16 import stacked  # noqa: E402

KIND = sys.argv[1] if len(sys.argv) > 1 else "2349"
PROOFS = int(sys.argv[2]) if len(sys.argv) > 2 else 1  # > 1: back-to-back proofs (rocprofv3 lane timeline)


def mem(tag):
    f, t = torch.cuda.mem_get_info(0)
    print(f"[mem] {tag}: used {(t - f) / 1e9:.1f} GB free {f / 1e9:.1f} GB", flush=True)


ctx = fg.Context(0)
mem("ctx")
if KIND == "stacked":
    c = stacked.StackedCircuit(11, 18, 1 << 30, 8, 8, 0)
else:
    c = stacked.FallbackPoStCircuit(int(KIND), 10, 1 << 30, 8, 8, 0)
gc_ = c.load(ctx)
mem(f"circuit loaded (n={c.num_constraints} n_a={gc_.n_a} n_b={gc_.n_b} nnz={gc_.nnz})")
pk = fg.generate_random_parameters(ctx, gc_, [3, 5, 7, 11, 13])
ctx.synchronize()
mem(f"key generated {pk.msm_info()}")
if KIND == "stacked":
    slots = stacked.slots_of(c, stacked.synthetic_instance(ctx, c, seed=1))
else:
    _, sectors = stacked.synthetic_post_instance(ctx, c, seed=1)
    slots = stacked.post_slots(c, sectors)
sd = torch.from_numpy(np.frombuffer(slots, dtype=np.uint8).copy()).cuda()
z = torch.empty(32 * c.num_vars, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
c.witness_dev(ctx, sd.data_ptr(), z.data_ptr())
ctx.synchronize()
mem("witness")
t = time.perf_counter()
try:
    for k in range(PROOFS):
        t = time.perf_counter()
        proof = fg.prove(ctx, pk, gc_, z.data_ptr())
        ctx.synchronize()
        print(f"proof {k}: {time.perf_counter() - t:.3f} s", flush=True)
finally:
    mem("after prove")
