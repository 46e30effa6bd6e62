"""Debug helper: run small MSMs / NTT through the C ABI, one step at a time (use with
AMD_SERIALIZE_KERNEL=3 HIP_LAUNCH_BLOCKING=1 to localise device faults)."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "crypto3-fil-proofs_amd"), os.path.join(ROOT, "oracle")]
import fil_groth16 as fg
import oracle_py as o

ctx = fg.Context(0)
for n in [int(x) for x in (sys.argv[1:] or ["1", "8", "64"])]:
    rng = np.random.default_rng(n)
    k = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64); k[:, 3] &= np.uint64(2**62 - 1)
    s = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64); s[:, 3] &= np.uint64(2**62 - 1)
    bases = o.g1_fixed_base(k.tobytes())
    print("n", n, "c", fg.msm_window_bits(n), flush=True)
    got = ctx.msm_g1(bases, s.tobytes())
    print("  gpu ok", got == o.msm_g1(bases, s.tobytes()), flush=True)
for n in [int(x) for x in (sys.argv[1:] or ["1", "8", "64"])]:
    rng = np.random.default_rng(n)
    k = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64); k[:, 3] &= np.uint64(2**62 - 1)
    s = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64); s[:, 3] &= np.uint64(2**62 - 1)
    bases = o.g2_fixed_base(k.tobytes())
    print("g2 n", n, flush=True)
    got = ctx.msm_g2(bases, s.tobytes())
    print("  gpu ok", got == o.msm_g2(bases, s.tobytes()), flush=True)
