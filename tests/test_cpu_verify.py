"""CPU: the product-side Groth16 verifier (mi_groth16_verify / _batch, host code in verify.hip --
bellman verify_proof semantics, the C2 self-check of api/seal.hpp:310-313) against the golden
proofs and oracle-made proofs, plus pairing bilinearity and the latency mode's share assembly
(mi_groth16_assemble).  No device is needed."""
import random

import pytest

import circuits
import fil_groth16 as fg

R = fg.FR_MODULUS


def _case(oracle, name):
    if name.startswith("random"):
        _, seed, rows = name.split("_")
        n_in, n_aux, rws, z = circuits.random_circuit(int(seed), int(rows))
    else:
        n_in, n_aux, rws, z = circuits.toy_chain(1022)
    oc = oracle.OracleCircuit(len(rws), n_in, n_aux, circuits.to_csr(rws))
    op = oracle.OracleParams(oc, circuits.toxic())
    ex = op.export()
    zb = circuits.z_bytes(z)
    return op, ex, zb, n_in


@pytest.mark.parametrize("name", ["random_11_24", "random_12_60", "toy_chain_1022"])
def test_verify_golden(oracle, golden, name):
    op, ex, zb, n_in = _case(oracle, name)
    proof = bytes.fromhex(golden["groth16"][name]["proof"])
    inputs = zb[32:32 * n_in]  # public inputs without ONE
    assert fg.verify(ex["vk"], ex["ic"], inputs, proof)
    # wrong public input
    bad_in = bytearray(inputs)
    bad_in[0] ^= 1
    assert not fg.verify(ex["vk"], ex["ic"], bytes(bad_in), proof)
    # A and C swapped (both valid G1 encodings)
    swapped = proof[144:192] + proof[48:144] + proof[0:48]
    assert not fg.verify(ex["vk"], ex["ic"], inputs, swapped)


def test_verify_rejects_bad_encodings(oracle, golden):
    op, ex, zb, n_in = _case(oracle, "random_11_24")
    proof = bytearray.fromhex(golden["groth16"]["random_11_24"]["proof"])
    inputs = zb[32:32 * n_in]
    p1 = bytearray(proof)
    p1[0] &= 0x7F  # clear the compression flag
    with pytest.raises(fg.FilGpuError) as e:
        fg.verify(ex["vk"], ex["ic"], inputs, bytes(p1))
    assert e.value.code == -3  # MI_ERR_INVALID_POINT
    p2 = bytearray(proof)
    p2[47] ^= 1  # x of A changed: no longer decodes to a subgroup point, or a different point
    try:
        assert not fg.verify(ex["vk"], ex["ic"], inputs, bytes(p2))
    except fg.FilGpuError as e2:
        assert e2.code == -3
    big = (R + 1).to_bytes(32, "little")
    with pytest.raises(fg.FilGpuError) as e3:
        fg.verify(ex["vk"], ex["ic"], big + inputs[32:], bytes(proof))
    assert e3.value.code == -1  # non-canonical public input


def test_verify_batch(oracle):
    op, ex, zb, n_in = _case(oracle, "random_11_24")
    inputs = zb[32:32 * n_in]
    rng = random.Random(3)
    proofs = [op.prove(zb, rng.randrange(R), rng.randrange(R))[0] for _ in range(4)]
    seed = bytes(range(32))
    assert fg.verify_batch(ex["vk"], ex["ic"], [inputs] * 4, proofs, seed)
    assert fg.verify_batch(ex["vk"], ex["ic"], [], [], seed)
    bad = list(proofs)
    bad[2] = proofs[2][144:192] + proofs[2][48:144] + proofs[2][0:48]
    assert not fg.verify_batch(ex["vk"], ex["ic"], [inputs] * 4, bad, seed)
    wrong = inputs[:-32] + b"\x05" + bytes(31)
    assert not fg.verify_batch(ex["vk"], ex["ic"], [wrong] + [inputs] * 3, proofs, seed)
    # production mode: weights from getrandom() (bellman OsRng), no caller-chosen seed
    assert fg.verify_batch(ex["vk"], ex["ic"], [inputs] * 4, proofs)
    assert not fg.verify_batch(ex["vk"], ex["ic"], [inputs] * 4, bad)


def test_pairing_bilinear(oracle):
    g1, g2 = oracle.g1_generator(), oracle.g2_generator()
    a, b = 0x1234567, 0xABCDEF12345
    e_ab = fg.pairing(oracle.g1_mul(g1, a), oracle.g2_mul(g2, b))
    assert e_ab == fg.pairing(oracle.g1_mul(g1, a * b % R), g2)
    assert e_ab == fg.pairing(g1, oracle.g2_mul(g2, a * b % R))
    e1 = fg.pairing(g1, g2)
    one = bytes(47) + b"\x01" + bytes(48 * 11)
    assert e1 != one  # non-degenerate
    assert fg.pairing(oracle.g1_mul(g1, R - 1), g2) != e1


@pytest.mark.parametrize("world", [1, 3, 50])
def test_assemble_shares_matches_oracle(oracle, world):
    """mi_groth16_assemble (host): oracle shares of any split -- 50 ranks leave some slices empty --
    add up and blind to the oracle's proof."""
    import split_oracle

    n_in, n_aux, rows, z = circuits.random_circuit(72, 30)
    mats = circuits.to_csr(rows)
    P = oracle.OracleParams(oracle.OracleCircuit(len(rows), n_in, n_aux, mats), circuits.toxic())
    zb = circuits.z_bytes(z)
    sh = split_oracle.shares(oracle, P, n_in, n_aux, mats, zb, world)
    vk = P.export()["vk"]
    proof, raw = fg.assemble(vk, sh, 3, 4, want_raw=True)
    oproof, oraw, _ = P.prove(zb, 3, 4)
    assert proof == oproof and raw == oraw
    assert fg.assemble(vk, sh[::-1], 3, 4) == oproof  # order-free


def test_assemble_rejects_bad_shares(oracle):
    import split_oracle

    n_in, n_aux, rows, z = circuits.random_circuit(73, 20)
    mats = circuits.to_csr(rows)
    P = oracle.OracleParams(oracle.OracleCircuit(len(rows), n_in, n_aux, mats), circuits.toxic())
    sh = split_oracle.shares(oracle, P, n_in, n_aux, mats, circuits.z_bytes(z), 2)
    vk = P.export()["vk"]
    bad = bytearray(sh[0])
    bad[100] ^= 1  # L's x coordinate: off the curve
    with pytest.raises(fg.FilGpuError):
        fg.assemble(vk, [bytes(bad), sh[1]], 1, 2)
    with pytest.raises(ValueError):
        fg.assemble(vk, [], 1, 2)
    with pytest.raises(fg.FilGpuError):
        fg.assemble(vk, sh, fg.FR_MODULUS.to_bytes(32, "little"), 2)  # r >= r_mod
