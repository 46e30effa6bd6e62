"""CPU: the SDR labelling-witness oracle (oracle.cpp or_sha256 / or_sdr_labels) against the FIPS 180-2
SHA-256 known answers, hashlib, and tests/golden/sdr_golden.json; the Python mirror's
host-side helpers."""
import hashlib
import json
import os
import random

import pytest

import fil_groth16 as fg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "sdr_golden.json")))

# FIPS 180-2 appendix B.1 / B.2 and the empty message
FIPS = [(b"abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
        (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
         "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
        (b"", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855")]


@pytest.mark.parametrize("msg,digest", FIPS)
def test_oracle_sha256_fips(oracle, msg, digest):
    assert oracle.sha256(msg).hex() == digest


def test_oracle_sha256_lengths_vs_hashlib(oracle):
    rng = random.Random(1)
    for n in list(range(0, 130)) + [1247, 1248, 1249, 4096]:
        m = bytes(rng.randrange(256) for _ in range(n))
        assert oracle.sha256(m) == hashlib.sha256(m).digest(), n


def test_oracle_labels_match_golden(oracle):
    for c in GOLD["cases"]:
        par = b"".join(bytes.fromhex(p) for p in c["parents"])
        got = oracle.sdr_labels(bytes.fromhex(c["replica_id"]), [c["layer"]], [c["node"]], par, len(c["parents"]))
        assert got.hex() == c["label"], c


def test_oracle_labels_batch_and_refusal(oracle):
    rng = random.Random(2)
    rid = bytes(rng.randrange(256) for _ in range(32))
    n, np_ = 300, 14  # >= 256: the OpenMP branch
    layers = [rng.randrange(1, 12) for _ in range(n)]
    nodes = [rng.randrange(2 ** 35) for _ in range(n)]
    par = bytes(rng.randrange(256) for _ in range(32 * np_ * n))
    got = oracle.sdr_labels(rid, layers, nodes, par, np_)
    for i in (0, 17, 299):
        ps = [par[(i * np_ + k) * 32:(i * np_ + k + 1) * 32] for k in range(np_)]
        msg = rid + layers[i].to_bytes(4, "big") + nodes[i].to_bytes(8, "big") + bytes(20)
        msg += b"".join(ps[k % np_] for k in range(37))
        d = bytearray(hashlib.sha256(msg).digest())
        d[31] &= 0x3F
        assert got[32 * i:32 * i + 32] == bytes(d)
    with pytest.raises(ValueError):
        oracle.sdr_labels(rid, [1], [1], bytes(32 * 38), 38)


def test_labels_are_canonical_fr(oracle):
    c = GOLD["cases"][0]
    lab = bytes.fromhex(c["label"])
    assert int.from_bytes(lab, "little") < fg.FR_MODULUS and lab[31] < 0x40


def test_repeat_parents_and_encode():
    ps = [bytes([i]) * 32 for i in range(14)]
    full = fg.sdr.repeat_parents(ps)
    assert len(full) == 37 and full[:14] == ps and full[14:28] == ps and full[28:] == ps[:9]
    assert fg.sdr.repeat_parents([]) == []
    r = fg.FR_MODULUS
    assert fg.sdr.encode((r - 1).to_bytes(32, "little"), (5).to_bytes(32, "little")) == (4).to_bytes(32, "little")
    with pytest.raises(ValueError):
        fg.sdr.encode(r.to_bytes(32, "little"), bytes(32))


# Reference-held tree D vectors: compute_comm_d of an empty 2048-byte and 128-byte sector
# (libs/filecoin/test/pieces.cpp:86-95): 64 / 4 zero leaves, SHA-256 node hash, byte 31 &= 0x3f.
COMM_D_EMPTY = {
    64: bytes([252, 126, 146, 130, 150, 229, 22, 250, 173, 233, 134, 178, 143, 146, 212, 74,
               79, 36, 185, 53, 72, 82, 35, 55, 106, 121, 144, 39, 188, 24, 248, 51]),
    4: bytes.fromhex("3731bb99ac689f66eef5973e4a94da188f4ddcae580724fc6f3fd60dfd488333"),
}


@pytest.mark.parametrize("leaves", sorted(COMM_D_EMPTY))
def test_oracle_tree_d_root_matches_reference_comm_d(oracle, leaves):
    row = [bytes(32)] * leaves
    while len(row) > 1:
        nxt = []
        for i in range(0, len(row), 2):
            d = bytearray(oracle.sha256(row[i] + row[i + 1]))
            d[31] &= 0x3F
            nxt.append(bytes(d))
        row = nxt
    assert row[0] == COMM_D_EMPTY[leaves]
