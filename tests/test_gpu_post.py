"""GPU: the Fallback PoSt circuit witness, against the oracle and the
reference's partition size.

* Small partitions over fully built trees (oracle/stacked_instance.py generate_post): the GPU witness equals
  the oracle's synthesis (oracle/stacked_circuit.py fallback_post_circuit) variable for variable for 8-0-0,
  8-4-2 and 4-0-0 trees; it satisfies the library's R1CS on the device, its public inputs equal the
  compound's order, and it proves and pairing-verifies.
* The synthetic partition generator (fil_groth16.stacked.synthetic_post_instance: sparse trees R-last on the
  GPU, challenges by generate_leaf_challenge) yields witnesses the device check accepts, equal to the
  oracle's synthesis over the same openings.
* One 32 GiB Window PoSt partition (2349 sectors x 10 challenges over 2^30-node 8-8-0 trees: 125,279,217
  constraints, constants.hpp:85-89; BASELINE config 5's partition) and one 64 GiB partition (2300 x 10 over
  2^31-node 8-8-2 trees: 129,887,900 constraints): the witness satisfies every row on the device; the partition
  proves and pairing-verifies.
Variable order beyond the reference's counts is parity-unpinned (oracle header).
"""
import numpy as np
import pytest
import torch

import fil_groth16 as fg
from fil_groth16 import stacked

pytestmark = pytest.mark.gpu


def _oracle_z(inst, shape):
    import stacked_circuit as sc

    cs = sc.CS(with_constraints=False)
    sc.fallback_post_circuit(cs, inst, shape)
    return b"".join(v.to_bytes(32, "little") for v in cs.z())


def test_post_small_witness_prove_verify(ctx, oracle):
    import circuits
    import stacked_instance as si

    shape = (8, 0, 0)
    c = stacked.FallbackPoStCircuit(2, 2, 64, *shape)
    inst = si.generate_post(2, 2, 64, shape, seed=4)
    slots = stacked.post_slots(c, inst["sectors"])
    got = c.witness(ctx, slots)
    assert got == _oracle_z(inst, shape)
    pub = c.public_inputs(slots)
    assert pub == b"".join(v.to_bytes(32, "little") for v in si.post_public_inputs(inst))
    assert got[32:32 * c.num_inputs] == pub
    gc = c.load(ctx)
    zd = torch.from_numpy(np.frombuffer(got, dtype=np.uint8).copy()).cuda()
    assert stacked.circuit_check_dev(ctx, gc, zd.data_ptr()) == (0, None)
    bad = zd.clone()
    bad[32 * (c.num_vars - 7)] ^= 1
    assert stacked.circuit_check_dev(ctx, gc, bad.data_ptr())[0] > 0
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    vk, ic = pk.verifying_key()
    proof = fg.prove(ctx, pk, gc, zd.data_ptr())
    assert fg.verify(vk, ic, pub, proof)
    assert not fg.verify(vk, ic, pub[:32 * 2] + bytes(32) + pub[32 * 3:], proof)


@pytest.mark.parametrize("shape,nodes", [((8, 4, 2), 512), ((4, 0, 0), 64), ((2, 0, 0), 16)])
def test_post_shapes_witness_vs_oracle(ctx, oracle, shape, nodes):
    import stacked_instance as si

    c = stacked.FallbackPoStCircuit(2, 3, nodes, *shape, with_r1cs=False)
    inst = si.generate_post(2, 3, nodes, shape, seed=8)
    assert c.witness(ctx, stacked.post_slots(c, inst["sectors"])) == _oracle_z(inst, shape)


def test_post_synthetic_instance_satisfies(ctx, oracle):
    shape, nodes = (8, 8, 0), 1 << 30
    c = stacked.FallbackPoStCircuit(4, 10, nodes, *shape)
    _, sectors = stacked.synthetic_post_instance(ctx, c, seed=5)
    slots = stacked.post_slots(c, sectors)
    z = torch.empty(32 * c.num_vars, dtype=torch.uint8, device="cuda")
    sd = torch.from_numpy(np.frombuffer(slots, dtype=np.uint8).copy()).cuda()
    torch.cuda.synchronize()
    c.witness_dev(ctx, sd.data_ptr(), z.data_ptr())
    gc = c.load(ctx)
    assert stacked.circuit_check_dev(ctx, gc, z.data_ptr()) == (0, None)
    inst = {"sectors": sectors, "nodes": nodes, "shape": shape}
    assert z.cpu().numpy().tobytes() == _oracle_z(inst, shape)


def test_post_32gib_window_partition_prove_verify(ctx):
    """BASELINE config 5's partition on the real circuit: 2349 sectors x 10 challenges, 125,279,217
    constraints, domain 2^27.  Witness satisfied on the device, proof pairing-verified."""
    import time

    import circuits

    t0 = time.perf_counter()

    def note(what):
        print(f"[window-post] {what}: {time.perf_counter() - t0:.1f} s", flush=True)

    c = stacked.FallbackPoStCircuit(2349, 10, 1 << 30, 8, 8, 0)
    assert (c.num_constraints, c.num_inputs) == (125_279_217, 25_840)
    note(f"R1CS built ({c.info['r1cs_entries']} entries)")
    _, sectors = stacked.synthetic_post_instance(ctx, c, seed=10)
    slots = stacked.post_slots(c, sectors)
    note("synthetic partition")
    gc = c.load(ctx)
    assert gc.d == 1 << 27
    note("circuit loaded")
    sd = torch.from_numpy(np.frombuffer(slots, dtype=np.uint8).copy()).cuda()
    z = torch.empty(32 * c.num_vars, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    c.witness_dev(ctx, sd.data_ptr(), z.data_ptr())
    note("witness")
    assert stacked.circuit_check_dev(ctx, gc, z.data_ptr()) == (0, None)
    note("R1CS check")
    pub = c.public_inputs(slots)
    assert z[32:32 * c.num_inputs].cpu().numpy().tobytes() == pub
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    note("keygen")
    vk, ic = pk.verifying_key()
    proof = fg.prove(ctx, pk, gc, z.data_ptr())
    note("proof")
    assert fg.verify(vk, ic, pub, proof)
    del pk, gc, z
    torch.cuda.synchronize()


def test_post_64gib_window_partition_prove_verify(ctx):
    """The 64 GiB Window-PoSt partition (constants.hpp:85-89: 2300 sectors x 10 challenges over 2^31-node 8-8-2
    trees R-last, 129,887,900 constraints, domain 2^27): synthetic partition, witness satisfied on the device, key
    generated, proof pairing-verified.  The memory fallbacks of keygen and prove (out-of-memory releases and
    retries, mi_ctx_get_fallbacks) and the key's table state are printed for the record."""
    import json
    import time

    import circuits

    t0 = time.perf_counter()

    def note(what):
        print(f"[window-post-64] {what}: {time.perf_counter() - t0:.1f} s", flush=True)

    c = stacked.FallbackPoStCircuit(2300, 10, 1 << 31, 8, 8, 2)
    assert c.num_constraints == 129_887_900
    note(f"R1CS built ({c.info['r1cs_entries']} entries, {c.num_inputs} inputs)")
    _, sectors = stacked.synthetic_post_instance(ctx, c, seed=64)
    slots = stacked.post_slots(c, sectors)
    note("synthetic partition")
    gc = c.load(ctx)
    assert gc.d == 1 << 27
    sd = torch.from_numpy(np.frombuffer(slots, dtype=np.uint8).copy()).cuda()
    z = torch.empty(32 * c.num_vars, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    c.witness_dev(ctx, sd.data_ptr(), z.data_ptr())
    note("witness")
    assert stacked.circuit_check_dev(ctx, gc, z.data_ptr()) == (0, None)
    note("R1CS check")
    pub = c.public_inputs(slots)
    assert z[32:32 * c.num_inputs].cpu().numpy().tobytes() == pub
    ctx.reset_stats()
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    keygen_fb = ctx.fallbacks()
    note(f"keygen (fallbacks {keygen_fb}, tables {pk.table_state()})")
    vk, ic = pk.verifying_key()
    ctx.reset_stats()
    t1 = time.perf_counter()
    proof = fg.prove(ctx, pk, gc, z.data_ptr())
    dt = time.perf_counter() - t1
    prove_fb = ctx.fallbacks()
    note(f"proof {1e3 * dt:.0f} ms (fallbacks {prove_fb})")
    assert fg.verify(vk, ic, pub, proof)
    free_b, total_b = torch.cuda.mem_get_info()
    print("[window-post-64] record " + json.dumps({
        "constraints": c.num_constraints, "inputs": c.num_inputs, "domain": gc.d, "prove_ms": 1e3 * dt,
        "keygen_fallbacks": keygen_fb, "prove_fallbacks": prove_fb, "table_state": pk.table_state(),
        "device_free_gb": free_b / 1e9, "device_total_gb": total_b / 1e9, "verified": True}), flush=True)
    del pk, gc, z
    torch.cuda.synchronize()


# ------------------------------------------------------------------------------------------ Winning PoSt
def test_winning_post_small_witness_prove_verify(ctx, oracle):
    """Winning PoSt at the reference's shape (parameters.hpp:58-68: 66 sectors x 1 challenge, the one replica
    repeated as api/post.hpp:205-218 does) over a 64-node tree: GPU witness == oracle synthesis, satisfied on
    the device, proven and pairing-verified through generate_winning_post_proof."""
    import circuits
    import stacked_instance as si

    from fil_groth16.compound import generate_winning_post_proof

    shape = (8, 0, 0)
    c = stacked.WinningPoStCircuit(64, *shape)
    inst = si.generate_winning_post(64, shape, seed=12)
    slots = stacked.post_slots(c, inst["sectors"])
    got = c.witness(ctx, slots)
    assert got == _oracle_z(inst, shape)
    pub = c.public_inputs(slots)
    assert got[32:32 * c.num_inputs] == pub
    gc = c.load(ctx)
    zd = torch.from_numpy(np.frombuffer(got, dtype=np.uint8).copy()).cuda()
    assert stacked.circuit_check_dev(ctx, gc, zd.data_ptr()) == (0, None)
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    vk, ic = pk.verifying_key()
    proof = generate_winning_post_proof(ctx, pk, gc, 1, 1, got)
    assert len(proof) == 192 and fg.verify(vk, ic, pub, proof)
    assert fg.prove(ctx, pk, gc, zd.data_ptr(), 5, 6) == oracle.OracleParams(
        oracle.OracleCircuit(c.num_constraints, c.num_inputs, c.num_aux, c.csr()), circuits.toxic()).prove(got, 5, 6)[0]


def test_winning_post_32gib_prove_verify(ctx, oracle):
    """The 32 GiB Winning-PoSt partition (66 x 1 over a 2^30-node 8-8-0 tree R-last: 370,590 constraints,
    133 inputs, domain 2^19) from the synthetic generator: the GPU witness equals the oracle's synthesis over
    the same openings, satisfies every row on the device, and the proof pairing-verifies."""
    import circuits

    shape, nodes = (8, 8, 0), 1 << 30
    c = stacked.WinningPoStCircuit(nodes, *shape)
    assert (c.num_constraints, c.num_inputs) == (370_590, 133)
    _, sectors = stacked.synthetic_winning_post_instance(ctx, c, seed=13)
    assert len({s["comm_r"] for s in sectors}) == 1
    slots = stacked.post_slots(c, sectors)
    sd = torch.from_numpy(np.frombuffer(slots, dtype=np.uint8).copy()).cuda()
    z = torch.empty(32 * c.num_vars, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    c.witness_dev(ctx, sd.data_ptr(), z.data_ptr())
    gc = c.load(ctx)
    assert gc.d == 1 << 19
    assert stacked.circuit_check_dev(ctx, gc, z.data_ptr()) == (0, None)
    inst = {"sectors": sectors, "nodes": nodes, "shape": shape}
    assert z.cpu().numpy().tobytes() == _oracle_z(inst, shape)
    pub = c.public_inputs(slots)
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    vk, ic = pk.verifying_key()
    proof = fg.prove(ctx, pk, gc, z.data_ptr())
    assert fg.verify(vk, ic, pub, proof)
    assert not fg.verify(vk, ic, pub[:-32] + bytes(32), proof)
    # every lane layout and MSM path gives the same bytes: B_G1 on its own lane (default) or sharing B_G2's plan
    # (boolean-heavy B scalars: chunk trees of several levels over one plan), one lane, no window tables
    want = fg.prove(ctx, pk, gc, z.data_ptr(), 5, 6)
    assert fg.verify(vk, ic, pub, want)
    for knobs in ({"prove_b1_lane": 0}, {"prove_b1_lane": 1}, {"prove_lanes": 1}, {"msm_wt": 0}):
        with fg.tuned(**knobs):
            assert fg.prove(ctx, pk, gc, z.data_ptr(), 5, 6) == want, knobs
