"""CPU: the Fallback PoSt circuit (Window / Winning PoSt partitions).

* The reference sizes a Window PoSt partition by its constraint count: 2349 sectors of 32 GiB = 125,279,217
  constraints and 2300 sectors of 64 GiB = 129,887,900 (libs/filecoin/include/nil/filecoin/proofs/
  constants.hpp:85-89; 10 challenges per sector, trees R-last 8-8-0 over 2^30 nodes / 8-8-2 over 2^31).  The
  library's builder (mi_post_build) reproduces both, and so does the oracle's closed form.
* The oracle's restatement (oracle/stacked_circuit.py fallback_post_circuit) is satisfied by a fully built
  instance (oracle/stacked_instance.py generate_post) and its inputs equal the compound's public-input order.
* The builder's R1CS equals the oracle's row for row, coefficient for coefficient (2 sectors x 2 challenges,
  which covers the sector replication), and its public inputs equal the oracle's.
* generate_leaf_challenge (vanilla.hpp:398-411): the library helper equals the oracle's.
"""
import numpy as np
import pytest

import fil_groth16 as fg
from fil_groth16 import stacked

PINNED = [  # (sectors, challenges, nodes, (base, sub, top), constraints): constants.hpp:85-89
    (2349, 10, 1 << 30, (8, 8, 0), 125_279_217),
    (2300, 10, 1 << 31, (8, 8, 2), 129_887_900),
]


@pytest.mark.parametrize("sectors,challenges,nodes,shape,want", PINNED)
def test_builder_window_post_partition_sizes(sectors, challenges, nodes, shape, want):
    c = stacked.FallbackPoStCircuit(sectors, challenges, nodes, *shape, with_r1cs=False)
    assert c.num_constraints == want
    assert c.num_inputs == 1 + sectors * (1 + challenges)
    levels = stacked.tree_arities(nodes, *shape)
    assert c.info["poseidon_hashes"] == sectors * (1 + challenges * len(levels))


@pytest.mark.parametrize("sectors,challenges,nodes,shape,want", PINNED)
def test_oracle_closed_form_matches_reference(sectors, challenges, nodes, shape, want):
    import stacked_circuit as sc

    assert sc.post_constraints(sectors, challenges, sc.tree_levels(nodes, shape)) == want


@pytest.fixture(scope="module")
def small_post():
    import stacked_circuit as sc
    import stacked_instance as si

    inst = si.generate_post(2, 2, 64, (8, 0, 0), seed=4)
    cs = sc.CS()
    sc.fallback_post_circuit(cs, inst, (8, 0, 0))
    return inst, cs


def test_oracle_post_satisfied(small_post):
    import stacked_circuit as sc
    import stacked_instance as si

    inst, cs = small_post
    assert cs.is_satisfied() is None
    assert cs.inputs[1:] == si.post_public_inputs(inst)
    assert cs.n_constraints == sc.post_constraints(2, 2, [8, 8])
    cs.aux[3] ^= 1
    assert cs.is_satisfied() is not None
    cs.aux[3] ^= 1


def test_builder_post_r1cs_equals_oracle(small_post):
    inst, cs = small_post
    c = stacked.FallbackPoStCircuit(2, 2, 64, 8, 0, 0)
    assert (c.num_constraints, c.num_inputs, c.num_aux) == (cs.n_constraints, len(cs.inputs), len(cs.aux))
    mats, ocsr = c.csr(), cs.to_csr()
    for m in range(3):
        rp, col, co = mats[m]
        orp, ocol, oco = ocsr[m]
        assert np.array_equal(rp, np.asarray(orp, dtype=np.uint64)), m
        assert np.array_equal(col, np.asarray(ocol, dtype=np.uint32)), m
        assert co.tobytes() == b"".join(int(k).to_bytes(32, "little") for k in oco), m
    slots = stacked.post_slots(c, inst["sectors"])
    assert c.public_inputs(slots) == b"".join(v.to_bytes(32, "little") for v in cs.inputs[1:])


def test_post_sub_top_counts():
    """base-only, 8-2, 8-4-2 and 4-ary trees: the builder's count equals the oracle's synthesis"""
    import stacked_circuit as sc
    import stacked_instance as si

    for shape, nodes in (((4, 0, 0), 64), ((8, 2, 0), 128), ((8, 4, 2), 512), ((2, 0, 0), 16)):
        inst = si.generate_post(1, 3, nodes, shape, seed=6)
        cs = sc.CS(with_constraints=False)
        sc.fallback_post_circuit(cs, inst, shape)
        c = stacked.FallbackPoStCircuit(1, 3, nodes, *shape, with_r1cs=False)
        assert (c.num_constraints, c.num_inputs) == (cs.n_constraints, len(cs.inputs)), shape


def test_leaf_challenges_and_padding():
    import stacked_instance as si

    for sid, k in ((7, 0), (2 ** 39 + 5, 13), (1, 2 ** 40)):
        assert stacked.generate_leaf_challenge(12345, sid, k, 1 << 30) == si.generate_leaf_challenge(12345, sid, k,
                                                                                                        1 << 30)
    inst = si.generate_post(1, 2, 64, (8, 0, 0), seed=9)
    c = stacked.FallbackPoStCircuit(3, 2, 64, 8, 0, 0, with_r1cs=False)
    slots = stacked.post_slots(c, inst["sectors"])  # one real sector, padded to three by repetition
    one = len(slots) // 3
    assert slots[:one] == slots[one:2 * one] == slots[2 * one:]
    with pytest.raises(ValueError):
        stacked.post_slots(c, inst["sectors"] * 4)
    bad = bytearray(slots)
    bad[32 * 3] = 64  # challenged index >= nodes
    with pytest.raises(fg.FilGpuError, match="node index"):
        c.public_inputs(bytes(bad))


def test_builder_refuses_bad_post_shapes():
    for args in [(0, 1, 64, 8, 0, 0), (1, 0, 64, 8, 0, 0), (1, 1, 48, 8, 0, 0), (1, 1, 64, 3, 0, 0)]:
        with pytest.raises(fg.FilGpuError):
            stacked.FallbackPoStCircuit(*args, with_r1cs=False)


# ------------------------------------------------------------------------------------------ Winning PoSt
def test_winning_post_setup_params():
    """proofs/parameters.hpp:58-68: 66 challenges over 1 sector -> 66 circuit sectors x 1 challenge"""
    import stacked_instance as si

    for cc, sc, want in ((66, 1, (66, 1)), (66, 2, (33, 2)), (66, 66, (1, 66)), (10, 5, (2, 5))):
        assert stacked.winning_post_setup_params(cc, sc) == want
        assert si.winning_post_setup_params(cc, sc) == want
    for cc, sc in ((66, 4), (66, 0), (0, 1)):
        with pytest.raises(ValueError):
            stacked.winning_post_setup_params(cc, sc)
    assert (stacked.WINNING_POST_CHALLENGE_COUNT, stacked.WINNING_POST_SECTOR_COUNT) == (66, 1)
    assert stacked.winning_post_sectors(["r"], 3) == ["r"] * 3
    assert stacked.winning_post_sectors(["a", "b"], 2) == ["a", "b", "a", "b"]


def test_builder_winning_post_32gib_shape():
    """The 32 GiB Winning-PoSt circuit: 66 sectors x 1 challenge over 2^30-node 8-8-0 trees R-last.  Per
    sector 1 + 311 + 1, per challenge 10 levels x (3 + 22 + 505) + 2: 66 x 5,615 = 370,590 constraints;
    inputs ONE + 66 x (comm_r, challenge) = 133 (against 1 + 1 x 67 = 68 for the 1 x 66 shape)."""
    import stacked_circuit as sc

    c = stacked.WinningPoStCircuit(1 << 30, 8, 8, 0, with_r1cs=False)
    assert (c.sectors, c.challenges) == (66, 1)
    assert c.num_constraints == 370_590 == sc.post_constraints(66, 1, sc.tree_levels(1 << 30, (8, 8, 0)))
    assert c.num_inputs == 133
    assert c.info["poseidon_hashes"] == 66 * (1 + 10)
    # the domain the prover takes: constraints + inputs rows -> 2^19
    assert (c.num_constraints + c.num_inputs - 1).bit_length() == 19


def test_builder_winning_post_r1cs_equals_oracle():
    """The builder's Winning-PoSt R1CS equals the oracle's synthesis of generate_winning_post's layout, row for row;
    the public inputs are every sector slot's comm_r (the one replica's) then its challenged leaf."""
    import stacked_circuit as sc
    import stacked_instance as si

    inst = si.generate_winning_post(64, (8, 0, 0), seed=12)
    assert len(inst["sectors"]) == 66 and all(len(s["challenges"]) == 1 for s in inst["sectors"])
    assert len({s["comm_r"] for s in inst["sectors"]}) == 1
    cs = sc.CS()
    sc.fallback_post_circuit(cs, inst, (8, 0, 0))
    assert cs.is_satisfied() is None
    c = stacked.WinningPoStCircuit(64, 8, 0, 0)
    assert (c.num_constraints, c.num_inputs, c.num_aux) == (cs.n_constraints, len(cs.inputs), len(cs.aux))
    mats, ocsr = c.csr(), cs.to_csr()
    for m in range(3):
        rp, col, co = mats[m]
        orp, ocol, oco = ocsr[m]
        assert np.array_equal(rp, np.asarray(orp, dtype=np.uint64)), m
        assert np.array_equal(col, np.asarray(ocol, dtype=np.uint32)), m
        assert co.tobytes() == b"".join(int(k).to_bytes(32, "little") for k in oco), m
    slots = stacked.post_slots(c, inst["sectors"])
    assert c.public_inputs(slots) == b"".join(v.to_bytes(32, "little") for v in cs.inputs[1:])
    assert cs.inputs[1:] == si.post_public_inputs(inst)
