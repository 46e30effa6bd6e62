"""GPU: several resident proving keys on one device, as the reference's parameter memo holds them
(GROTH_PARAM_MEMORY_CACHE keeps STACKED[..], WINNING_POST[..] and WINDOW_POST[..] params side by side,
libs/filecoin/include/nil/filecoin/proofs/caches.hpp:48-116).

The 32 GiB stacked-PoRep key (130,278,541 constraints, generated first, with its 2^128 split tables while HBM
is free) and the 32 GiB Window-PoSt key (125,279,217 constraints) live in one context.  The second key's
generation and the Window-PoSt proof's working set (~109 GB) do not fit beside the first key with its tables;
an allocation that fails makes the library release the split tables of the keys on the device that no one is
using (and the context's idle scratch) and run the step again (prover.hip srs_generate / groth16_sums).  Both circuits prove and pairing-verify, and the stacked proof made after its tables
were released (GLV split) is byte-identical to the one made with them.  The same is checked once more with the
failure forced (mi_ctx_inject_oom), so the equality holds whether or not the natural failure happened.
"""
import json
import os

import numpy as np
import pytest
import torch

import fil_groth16 as fg
from fil_groth16 import stacked

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_32gib_keys_in_one_context(tune):
    import time

    import circuits

    t0 = time.perf_counter()
    log = {}

    def note(what):
        free, total = torch.cuda.mem_get_info(0)
        log[what] = {"t_s": round(time.perf_counter() - t0, 1), "used_gb": round((total - free) / 1e9, 1),
                     "free_gb": round(free / 1e9, 1)}
        print(f"[two-keys] {what}: {log[what]}", flush=True)

    c = fg.Context(0)

    def wit(circ, slots):
        sd = torch.from_numpy(np.frombuffer(slots, dtype=np.uint8).copy()).cuda()
        z = torch.empty(32 * circ.num_vars, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        circ.witness_dev(c, sd.data_ptr(), z.data_ptr())
        return z

    try:
        sc = stacked.StackedCircuit(11, 18, 1 << 30, 8, 8, 0)
        s_slots = stacked.slots_of(sc, stacked.synthetic_instance(c, sc, seed=32))
        pc = stacked.FallbackPoStCircuit(2349, 10, 1 << 30, 8, 8, 0)
        _, sectors = stacked.synthetic_post_instance(c, pc, seed=10)
        p_slots = stacked.post_slots(pc, sectors)
        pub1, pub2 = sc.public_inputs(s_slots), pc.public_inputs(p_slots)
        note("circuits built, instances made")
        g1 = sc.load(c)
        k1 = fg.generate_random_parameters(c, g1, circuits.toxic(1))
        assert k1.msm_info()["split_tables"]
        vk1, ic1 = k1.verifying_key()
        z1 = wit(sc, s_slots)
        p1 = fg.prove(c, k1, g1, z1.data_ptr(), 5, 6)  # with the 2^128 tables
        assert fg.verify(vk1, ic1, pub1, p1)
        note("stacked key (split tables) + proof")
        g2 = pc.load(c)
        c.reset_stats()
        k2 = fg.generate_random_parameters(c, g2, circuits.toxic(2))
        log["keygen_fallbacks"] = c.fallbacks()
        note(f"window key {k2.msm_info()}, keygen fallbacks {log['keygen_fallbacks']}, stacked key "
             f"{k1.msm_info()}")
        vk2, ic2 = k2.verifying_key()
        z2 = wit(pc, p_slots)
        c.reset_stats()
        p2 = fg.prove(c, k2, g2, z2.data_ptr(), 7, 8)
        assert fg.verify(vk2, ic2, pub2, p2)
        fb = c.fallbacks()
        note(f"window proof, fallbacks {fb}")
        p1b = fg.prove(c, k1, g1, z1.data_ptr(), 5, 6)
        assert p1b == p1
        note(f"stacked proof again (tables {k1.msm_info()['split_tables']}): byte-identical")
        c.inject_oom(-1)
        c.reset_stats()
        p1c = fg.prove(c, k1, g1, z1.data_ptr(), 5, 6)
        p2c = fg.prove(c, k2, g2, z2.data_ptr(), 7, 8)
        assert c.fallbacks()["oom_retries"] == 2
        c.inject_oom(0)
        assert p1c == p1 and p2c == p2
        assert not k1.msm_info()["split_tables"]
        note("forced prove-time fallback: both proofs byte-identical")
        log["natural_fallback"] = fb
        out = os.path.join(ROOT, "gpurun_out")
        if os.path.isdir(out):
            with open(os.path.join(out, "two_keys_memory.json"), "w") as f:
                json.dump(log, f, indent=1)
        del z1, z2, k1, k2, g1, g2
        torch.cuda.synchronize()
    finally:
        c.close()
