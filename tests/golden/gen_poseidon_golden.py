"""Generates tests/golden/poseidon_golden.json from oracle/poseidon_ref.py (TEST INFRASTRUCTURE).

PARITY UNPINNED: the reference holds no Poseidon vector (its crypto3 hash submodule is empty); these
fixtures pin the restatement against regressions and give the GPU tests known answers.  Contents: per
arity, the first/last round constants and MDS corners, and digests of edge and seeded random inputs;
an arity-8 tree over 512 seeded leaves (root and cached rows digest); a 2-layer and an 11-layer
tree C over 64 seeded nodes (roots).
    python tests/golden/gen_poseidon_golden.py
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import poseidon_ref as P  # noqa: E402


def seeded(seed, n):
    rng = random.Random(seed)
    return [rng.randrange(P.R) for _ in range(n)]


def digest_rows(vals):
    return hashlib.sha256(b"".join(P.fr_to_bytes(v) for v in vals)).hexdigest()


def main():
    out = {"r": hex(P.R), "sbox_field": P.SBOX_FIELD, "arities": {}}
    for a in (2, 4, 8, 11):
        h = P.poseidon(a)
        cases = [[0] * a, [P.R - 1] * a, list(range(1, a + 1))] + [seeded(1000 + a * 10 + k, a) for k in range(3)]
        out["arities"][str(a)] = {
            "t": h.t, "r_f": h.r_f, "r_p": h.r_p,
            "rc_first": hex(h.rc[0]), "rc_last": hex(h.rc[-1]), "mds_00": hex(h.m[0][0]), "mds_last": hex(h.m[-1][-1]),
            "cases": [{"in": [hex(x) for x in xs], "out": hex(h.hash(xs))} for xs in cases],
        }
    leaves = seeded(7, 512)
    rows = P.merkle_rows(leaves, 8)
    out["tree8_512"] = {"seed": 7, "root": hex(rows[-1][0]), "rows_sha256": digest_rows(P.tree_data(leaves, 8, 0)),
                        "rows_discard2_sha256": digest_rows(P.tree_data(leaves, 8, 2))}
    for layers in (2, 11):
        labs = [seeded(100 + l, 64) for l in range(layers)]
        base = P.hash_columns(labs)
        out[f"tree_c_{layers}x64"] = {"seed": 100, "base_sha256": digest_rows(base),
                                      "root": hex(P.merkle_rows(base, 8)[-1][0])}
    with open(os.path.join(HERE, "poseidon_golden.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
