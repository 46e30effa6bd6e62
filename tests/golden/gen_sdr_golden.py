"""Generates tests/golden/sdr_golden.json: SDR labelling-witness vectors.

Independent of oracle/: the label is computed with Python's hashlib SHA-256 over the message the reference
hashes for a LabelingProof (porep/stacked/vanilla/detail/processing/naive/labelling_proof.hpp:46-60,
create_label.hpp:49-77): replica_id || u32_be(layer) || u64_be(node) || 0^20 || parents repeated cyclically
to 37 (vanilla/proof.hpp:233-237), byte 31 &= 0x3f.  SHA-256 itself is pinned by the FIPS 180-2 vectors in
tests/test_cpu_sdr.py; the message layout is parity unpinned (the reference holds no label vector).
Run: python tests/golden/gen_sdr_golden.py
"""
import hashlib
import json
import os
import random

TOTAL_PARENTS = 37


def label(replica_id: bytes, layer: int, node: int, parents: list) -> bytes:
    msg = replica_id + layer.to_bytes(4, "big") + node.to_bytes(8, "big") + bytes(20)
    if parents:
        msg += b"".join(parents[k % len(parents)] for k in range(TOTAL_PARENTS))
    d = bytearray(hashlib.sha256(msg).digest())
    d[31] &= 0x3F
    return bytes(d)


def main():
    rng = random.Random(0x5D12)
    cases = []
    shapes = [(1, 0, 0), (1, 1, 6), (2, 7, 14), (11, 2 ** 30 - 1, 14), (3, 2 ** 40 + 3, 37), (5, 12, 1),
              (2, 99, 13), (0xFFFFFFFF, 2 ** 64 - 1, 2)]
    for layer, node, n_par in shapes:
        rid = bytes(rng.randrange(256) for _ in range(32))
        par = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(n_par)]
        cases.append({"replica_id": rid.hex(), "layer": layer, "node": node,
                      "parents": [p.hex() for p in par], "label": label(rid, layer, node, par).hex()})
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sdr_golden.json")
    with open(out, "w") as f:
        json.dump({"generator": "tests/golden/gen_sdr_golden.py (hashlib)", "cases": cases}, f, indent=1)


if __name__ == "__main__":
    main()
