"""GPU: the stacked-PoRep circuit witness, against the oracle and the reference's counts.

* The reference test shape (2 layers, 1 challenge, 8 nodes, Poseidon base 8: 1,199,620 constraints, 22
  inputs; libs/storage/test/porep/stacked/circuit/proof.cpp:145-147): the GPU witness of a fully built replica
  instance (oracle/stacked_instance.py) equals the oracle's synthesis (oracle/stacked_circuit.py) variable for
  variable, satisfies the library's R1CS on the device, its public inputs equal generate_public_inputs, and it
  proves with the library's prover and pairing-verifies.
* The other reference shapes (base 2, 8-4, 8-4-2) and a 2-challenge partition: GPU witness == oracle witness.
* The synthetic instance generator (sparse trees, labels from the GPU label kernel) yields satisfied witnesses.
* The 32 GiB shape (11 layers, 18 challenges, 2^30 nodes, 8-8 trees: 130,278,541 constraints): the GPU
  witness of a synthetic partition satisfies every constraint on the device, and the partition proves and
  pairing-verifies (BASELINE config 4 on the real circuit).
Parity of the variable layout is unpinned beyond the reference's counts (oracle header).
"""
import numpy as np
import pytest
import torch

import fil_groth16 as fg
from fil_groth16 import stacked

pytestmark = pytest.mark.gpu

SHAPES = {  # (base, sub, top), nodes = 8 x base-tree count; reference constraint count at 2 layers, 1 challenge
    "base_8": ((8, 0, 0), 8, 1_199_620),
    "base_2": ((2, 0, 0), 8, 1_206_212),
    "sub_8_4": ((8, 4, 0), 32, 1_296_576),
    "top_8_4_2": ((8, 4, 2), 64, 1_346_982),
}


def _oracle_z(inst, layers, nodes, shape):
    import stacked_circuit as sc

    cs = sc.CS(with_constraints=False)
    sc.stacked_circuit(cs, inst, layers, nodes, shape)
    return b"".join(v.to_bytes(32, "little") for v in cs.z()), cs


def test_stacked_reference_shape_witness_prove_verify(ctx, oracle):
    import circuits
    import stacked_instance as si

    shape, nodes, count = SHAPES["base_8"]
    c = stacked.StackedCircuit(2, 1, nodes, *shape)
    assert (c.num_constraints, c.num_inputs) == (count, 22)
    inst = si.generate(nodes, 2, shape, 1, seed=3)
    slots = stacked.slots_of(c, inst)
    want, cs = _oracle_z(inst, 2, nodes, shape)
    got = c.witness(ctx, slots)
    assert got == want
    pub = c.public_inputs(slots)
    assert pub == b"".join(v.to_bytes(32, "little") for v in si.public_inputs(inst))
    assert got[32:32 * c.num_inputs] == pub
    gc = c.load(ctx)
    zd = torch.from_numpy(np.frombuffer(got, dtype=np.uint8).copy()).cuda()
    assert stacked.circuit_check_dev(ctx, gc, zd.data_ptr()) == (0, None)
    bad = zd.clone()
    bad[32 * (c.num_vars - 5)] ^= 1  # flip one bit of a late variable: the device check must notice
    assert stacked.circuit_check_dev(ctx, gc, bad.data_ptr())[0] > 0
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    vk, ic = pk.verifying_key()
    proof = fg.prove(ctx, pk, gc, zd.data_ptr())
    assert fg.verify(vk, ic, pub, proof)
    assert not fg.verify(vk, ic, bytes(32) + pub[32:], proof)


@pytest.mark.parametrize("name", ["base_2", "sub_8_4", "top_8_4_2"])
def test_stacked_reference_shapes_witness_vs_oracle(ctx, oracle, name):
    import stacked_instance as si

    shape, nodes, count = SHAPES[name]
    c = stacked.StackedCircuit(2, 1, nodes, *shape, with_r1cs=False)
    assert c.num_constraints == count
    inst = si.generate(nodes, 2, shape, 1, seed=7)
    assert c.witness(ctx, stacked.slots_of(c, inst)) == _oracle_z(inst, 2, nodes, shape)[0]


def test_stacked_two_challenges_witness_and_check(ctx, oracle):
    import stacked_instance as si

    shape, nodes = (8, 0, 0), 8
    c = stacked.StackedCircuit(2, 2, nodes, *shape)
    inst = si.generate(nodes, 2, shape, 2, seed=11)
    got = c.witness(ctx, stacked.slots_of(c, inst))
    assert got == _oracle_z(inst, 2, nodes, shape)[0]
    gc = c.load(ctx)
    zd = torch.from_numpy(np.frombuffer(got, dtype=np.uint8).copy()).cuda()
    assert stacked.circuit_check_dev(ctx, gc, zd.data_ptr()) == (0, None)


def test_stacked_synthetic_instance_satisfies(ctx, oracle):
    shape, nodes = (8, 8, 0), 64
    c = stacked.StackedCircuit(11, 2, nodes, *shape)
    inst = stacked.synthetic_instance(ctx, c, seed=5)
    slots = stacked.slots_of(c, inst)
    z = torch.empty(32 * c.num_vars, dtype=torch.uint8, device="cuda")
    sd = torch.from_numpy(np.frombuffer(slots, dtype=np.uint8).copy()).cuda()
    torch.cuda.synchronize()
    c.witness_dev(ctx, sd.data_ptr(), z.data_ptr())
    gc = c.load(ctx)
    assert stacked.circuit_check_dev(ctx, gc, z.data_ptr()) == (0, None)
    assert z.cpu().numpy().tobytes() == _oracle_z(inst, 11, nodes, shape)[0]


def test_stacked_refuses_bad_instances(ctx):
    import stacked_instance as si

    shape, nodes = (8, 0, 0), 8
    c = stacked.StackedCircuit(2, 1, nodes, *shape, with_r1cs=False)
    slots = bytearray(stacked.slots_of(c, si.generate(nodes, 2, shape, 1, seed=3)))
    s = c.info["stride"]
    bad = bytearray(slots)
    bad[32 * 5] = nodes  # challenge index >= nodes
    with pytest.raises(fg.FilGpuError, match="node index"):
        c.witness(ctx, bytes(bad))
    bad = bytearray(slots)
    bad[32 * 6:32 * 7] = fg.FR_MODULUS.to_bytes(32, "little")  # data leaf = r
    with pytest.raises(fg.FilGpuError, match="canonical"):
        c.witness(ctx, bytes(bad))
    assert s == c.info["slots"] - 5
    with pytest.raises(fg.FilGpuError):
        stacked.StackedCircuit(3, 1, nodes, *shape)  # column hash arity 3 does not exist


def test_stacked_32gib_partition_witness_prove_verify(ctx):
    """BASELINE config 4 on the real circuit: one 32 GiB PoRep partition (11 layers, 18 challenges, 2^30 nodes,
    tree C / R-last 8-8; 130,278,541 constraints, domain 2^27).  The GPU witness of a synthetic partition
    satisfies all rows on the device; the partition proves and pairing-verifies."""
    import time

    import circuits

    t0 = time.perf_counter()

    def note(what):
        print(f"[32GiB] {what}: {time.perf_counter() - t0:.1f} s", flush=True)

    c = stacked.StackedCircuit(11, 18, 1 << 30, 8, 8, 0)
    assert (c.num_constraints, c.num_inputs) == (130_278_541, 328)
    note(f"R1CS built ({c.info['r1cs_entries']} entries)")
    inst = stacked.synthetic_instance(ctx, c, seed=32)
    slots = stacked.slots_of(c, inst)
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
