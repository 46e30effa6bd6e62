"""CPU: the oracle (oracle/oracle.cpp) against the committed golden fixtures.

The fixtures come from tests/golden/pyref.py, an independent pure-Python restatement; every
Groth16 fixture was accepted by a pairing check when generated.  Published constants pinned:
the zcash encodings of the BLS12-381 generators and bellman's Fr::ROOT_OF_UNITY.
"""
import hashlib

import pytest

import circuits


def test_published_constants(oracle, golden):
    f = golden["field"]
    assert oracle.g1_compress(oracle.g1_generator()).hex() == f["g1_generator_compressed"]
    assert oracle.g2_compress(oracle.g2_generator()).hex() == f["g2_generator_compressed"]
    assert oracle.g1_generator().hex() == f["g1_generator_uncompressed"]
    assert oracle.g2_generator().hex() == f["g2_generator_uncompressed"]
    # group order r: (r-1) G + G = O (0x40 infinity flag)
    g = oracle.g1_generator()
    assert oracle.g1_add(oracle.g1_mul(g, oracle.R_MOD - 1), g)[0] == 0x40
    g2 = oracle.g2_generator()
    assert oracle.g2_add(oracle.g2_mul(g2, oracle.R_MOD - 1), g2)[0] == 0x40


def test_roots_of_unity(oracle, golden):
    import ctypes

    for k, hexv in golden["field"]["roots_of_unity"].items():
        b = ctypes.create_string_buffer(32)
        oracle.lib().or_fr_root_of_unity(int(k), b)
        assert b.raw.hex() == hexv
    b = ctypes.create_string_buffer(32)
    oracle.lib().or_fr_root_of_unity(32, b)
    assert int.from_bytes(b.raw, "little") == 0x16A2A19EDFE81F20D09B681922C813B4B63683508C2280B93829971F439F0D2B


def test_fr_arith(oracle, golden):
    import ctypes

    for a, b, c in golden["field"]["fr_mul"]:
        out = ctypes.create_string_buffer(32)
        oracle.lib().or_fr_mul(bytes.fromhex(a), bytes.fromhex(b), out)
        assert out.raw.hex() == c
    for a, ai in golden["field"]["fr_inv"]:
        out = ctypes.create_string_buffer(32)
        oracle.lib().or_fr_inv(bytes.fromhex(a), out)
        assert out.raw.hex() == ai


def test_ntt_golden(oracle, golden):
    for log_n, ent in golden["ntt"].items():
        inp = bytes.fromhex(ent["input"])
        for kind, name in enumerate(("fft", "ifft", "coset_fft", "icoset_fft")):
            assert oracle.ntt(inp, int(log_n), kind).hex() == ent[name]


def test_msm_golden(oracle, golden):
    m = golden["msm"]
    for f in (oracle.msm_g1, oracle.msm_g1_naive):
        assert f(bytes.fromhex(m["g1"]["bases"]), bytes.fromhex(m["g1"]["scalars"])).hex() == m["g1"]["result"]
    assert oracle.msm_g2(bytes.fromhex(m["g2"]["bases"]), bytes.fromhex(m["g2"]["scalars"])).hex() == m["g2"]["result"]


def _circ(name):
    if name.startswith("random"):
        _, seed, rows = name.split("_")
        return circuits.random_circuit(int(seed), int(rows))
    return circuits.toy_chain(1022)


@pytest.mark.parametrize("name", ["random_11_24", "random_12_60", "toy_chain_1022"])
def test_groth16_golden(oracle, golden, name):
    g = golden["groth16"][name]
    n_in, n_aux, rows, z = _circ(name)
    c = oracle.OracleCircuit(len(rows), n_in, n_aux, circuits.to_csr(rows))
    zb = circuits.z_bytes(z)
    assert c.satisfied(zb)
    P = oracle.OracleParams(c, circuits.toxic())
    assert [P.nh, P.nl, P.na, P.nb1, P.nb2] == g["query_sizes"] and P.d == g["d"]
    r, s = circuits.blinding()
    proof, raw, h = P.prove(zb, r, s, want_h=True)
    assert proof.hex() == g["proof"]
    assert raw.hex() == g["raw"]
    assert hashlib.sha256(h).hexdigest() == g["h_sha256"]
    assert P.trapdoor_check(zb, r, s, raw)
    ex = P.export()
    assert oracle.groth16_verify(ex["vk"], ex["ic"], zb[:32 * n_in], raw)
    # a tampered proof must fail both checks
    bad = bytearray(raw)
    bad[96:288] = oracle.g2_mul(oracle.g2_generator(), 12345)
    assert not P.trapdoor_check(zb, r, s, bytes(bad))
    assert not oracle.groth16_verify(ex["vk"], ex["ic"], zb[:32 * n_in], bytes(bad))
    # wrong public input must fail the pairing check
    wrong = bytearray(zb[:32 * n_in])
    wrong[32] ^= 1
    assert not oracle.groth16_verify(ex["vk"], ex["ic"], bytes(wrong), raw)


def test_params_roundtrip_from_queries(oracle):
    n_in, n_aux, rows, z = circuits.random_circuit(13, 50)
    c = oracle.OracleCircuit(len(rows), n_in, n_aux, circuits.to_csr(rows))
    P = oracle.OracleParams(c, circuits.toxic())
    Q = oracle.OracleParams(c, queries=P.export())
    zb = circuits.z_bytes(z)
    assert P.prove(zb, 3, 4)[0] == Q.prove(zb, 3, 4)[0]
