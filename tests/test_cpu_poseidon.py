"""CPU: Poseidon / tree-builder host logic -- no GPU compute.

* the library's host-derived constants (its own Grain LFSR + Cauchy MDS, mi_poseidon_constants) equal the
  independent restatement oracle/poseidon_ref.py, for every supported arity;
* the device arithmetic (9 x 29-bit lazy Fr, folded constants, sparse partial rounds; csrc/poseidon_math.h)
  compiled for the host equals the oracle's literal permutation on edge and random inputs;
* the oracle reproduces the committed fixtures (tests/golden/poseidon_golden.json);
* tree sizes follow get_merkle_tree_cache_size / default_rows_to_discard semantics.
PARITY UNPINNED: the reference holds no Poseidon vector (crypto3 hash submodule empty)."""
import json
import os
import random
import subprocess

import pytest

import fil_groth16 as fg
import poseidon_ref as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.parametrize("arity", [2, 4, 8, 11])
def test_library_constants_equal_oracle(arity):
    t, rf, rp, rc, mds = fg.tree.poseidon_constants(arity)
    ref = P.poseidon(arity)
    assert (t, rf, rp) == (ref.t, ref.r_f, ref.r_p)
    assert rc == ref.rc
    assert mds == ref.m
    assert all(mds[i][j] == mds[j][i] for i in range(t) for j in range(t))  # Cauchy 1/(i+j+t): symmetric


def test_unsupported_arity_rejected():
    with pytest.raises(fg.FilGpuError):
        fg.tree.poseidon_constants(3)


def test_oracle_matches_golden():
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "poseidon_golden.json")))
    assert int(g["r"], 16) == P.R
    for a, d in g["arities"].items():
        h = P.poseidon(int(a))
        assert hex(h.rc[0]) == d["rc_first"] and hex(h.rc[-1]) == d["rc_last"]
        for c in d["cases"]:
            assert hex(h.hash([int(x, 16) for x in c["in"]])) == c["out"]


@pytest.fixture(scope="module")
def host_poseidon(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    exe = str(tmp_path_factory.mktemp("pos") / "poseidon_check")
    subprocess.run([HIPCC, "-x", "hip", "--offload-host-only", "-std=c++17", "-O1", "-w", "-I",
                    os.path.join(ROOT, "crypto3-fil-proofs_amd", "csrc"),
                    os.path.join(ROOT, "tests", "host", "poseidon_check.cpp"), "-o", exe],
                   check=True, capture_output=True, timeout=600)
    return exe


def test_device_arithmetic_on_host_equals_oracle(host_poseidon):
    rng = random.Random(5)
    lines, want = [], []
    for a in (2, 4, 8, 11):
        cases = [[0] * a, [P.R - 1] * a, [1] + [0] * (a - 1)] + [[rng.randrange(P.R) for _ in range(a)] for _ in range(12)]
        for xs in cases:
            lines.append(" ".join([str(a)] + ["%x" % x for x in xs]))
            want.append("%064x" % P.poseidon(a).hash(xs))
    r = subprocess.run([host_poseidon], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == want


def test_tree_cache_size_semantics():
    # base row excluded, then the rows_to_discard lowest rows (merkletree get_merkle_tree_cache_size)
    assert fg.tree.get_merkle_tree_cache_size(8 ** 4, 8, 0) == 512 + 64 + 8 + 1
    assert fg.tree.get_merkle_tree_cache_size(8 ** 4, 8, 2) == 8 + 1
    assert fg.tree.get_merkle_tree_cache_size(2 ** 10, 2, 0) == 2 ** 10 - 1
    assert fg.tree.get_merkle_tree_cache_size(11 ** 2, 11, 1) == 1
    with pytest.raises(fg.FilGpuError):
        fg.tree.get_merkle_tree_cache_size(8 ** 3, 8, 3)  # would discard the root
    with pytest.raises(fg.FilGpuError):
        fg.tree.get_merkle_tree_cache_size(100, 8, 0)  # not a power of the arity
    assert fg.tree.default_rows_to_discard(8 ** 9, 8) == 2
    assert fg.tree.default_rows_to_discard(8, 8) == 0
    leaves = list(range(64))
    assert len(P.tree_data(leaves, 8, 0)) == fg.tree.get_merkle_tree_cache_size(64, 8, 0)
    assert len(P.tree_data(leaves, 8, 1)) == fg.tree.get_merkle_tree_cache_size(64, 8, 1)


def test_sparse_form_restatements_agree():
    """The oracle's own sparse-form derivation (poseidon_ref.sparse_form, independent of the library's C++)
    evaluates to the literal permutation, in Python and in the C oracle used as the CPU baseline."""
    import oracle_py

    rng = random.Random(9)
    for a in (2, 4, 8, 11):
        for _ in range(2):
            st = [P.poseidon(a).tag] + [rng.randrange(P.R) for _ in range(a)]
            assert P.permute_sparse(a, st) == P.poseidon(a).permute(st)
        xs = [rng.randrange(P.R) for _ in range(8 * a)]
        b = b"".join(P.fr_to_bytes(x) for x in xs)
        assert oracle_py.poseidon_hash_sparse(a, b) == oracle_py.poseidon_hash(a, b)
        assert fg.tree.to_ints(oracle_py.poseidon_hash(a, b)) == [P.poseidon(a).hash(xs[i * a:(i + 1) * a])
                                                                   for i in range(8)]
