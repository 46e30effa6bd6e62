"""GPU parity: Poseidon hash batches, TreeBuilder, ColumnTreeBuilder (tree C) and tree R-last through the
C ABI, bit-exact against the restatement oracle/poseidon_ref.py and tests/golden/poseidon_golden.json.
PARITY UNPINNED (no reference Poseidon vector); size-independent property at scale: every
sampled parent of a large device-built tree is the oracle hash of its children."""
import hashlib
import json
import os
import random

import numpy as np
import pytest
import torch

import fil_groth16 as fg
import poseidon_ref as P

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "poseidon_golden.json")))


def seeded(seed, n):
    rng = random.Random(seed)
    return [rng.randrange(P.R) for _ in range(n)]


def rows_sha(buf):
    return hashlib.sha256(bytes(buf)).hexdigest()


def ints(buf):
    return fg.tree.to_ints(buf)


@pytest.mark.parametrize("arity", [2, 4, 8, 11])
def test_poseidon_golden(ctx, arity):
    cases = GOLD["arities"][str(arity)]["cases"]
    pre = [int(x, 16) for c in cases for x in c["in"]]
    out = ints(fg.tree.poseidon_hash(ctx, arity, pre))
    assert out == [int(c["out"], 16) for c in cases]


@pytest.mark.parametrize("arity,n", [(2, 1), (2, 257), (8, 255), (11, 300), (4, 64)])
def test_poseidon_batch_vs_oracle(ctx, arity, n):
    pre = seeded(arity * 1000 + n, arity * n)
    out = ints(fg.tree.poseidon_hash(ctx, arity, pre))
    h = P.poseidon(arity)
    assert out == [h.hash(pre[i * arity:(i + 1) * arity]) for i in range(n)]


def test_poseidon_rejects_noncanonical(ctx):
    pre = [1] * 7 + [P.R]  # one entry == r
    with pytest.raises(fg.FilGpuError) as e:
        fg.tree.poseidon_hash(ctx, 8, pre)
    assert e.value.code == -1
    bad = b"\xff" * 32 + bytes(32)
    with pytest.raises(fg.FilGpuError):
        fg.tree.poseidon_hash(ctx, 2, bad)


def test_hash_single_column(ctx):
    col = seeded(3, 11)
    assert ints(fg.tree.hash_single_column(ctx, col)) == [P.poseidon(11).hash(col)]
    col2 = seeded(4, 2)
    assert ints(fg.tree.hash_single_column(ctx, col2)) == [P.poseidon(2).hash(col2)]


@pytest.mark.parametrize("discard", [0, 1, 2])
def test_tree_builder_golden(ctx, discard):
    leaves = seeded(GOLD["tree8_512"]["seed"], 512)
    tree = fg.tree.TreeBuilder(ctx, 8, discard).add_final_leaves(leaves)
    assert ints(tree) == P.tree_data(leaves, 8, discard)
    if discard == 0:
        assert rows_sha(tree) == GOLD["tree8_512"]["rows_sha256"]
        assert ints(tree)[-1] == int(GOLD["tree8_512"]["root"], 16)
    if discard == 2:
        assert rows_sha(tree) == GOLD["tree8_512"]["rows_discard2_sha256"]


@pytest.mark.parametrize("arity,n", [(2, 256), (4, 256), (11, 121)])
def test_tree_builder_other_arities(ctx, arity, n):
    leaves = seeded(arity, n)
    assert ints(fg.tree.TreeBuilder(ctx, arity).add_final_leaves(leaves)) == P.tree_data(leaves, arity, 0)


@pytest.mark.parametrize("layers", [2, 11])
def test_tree_c_golden(ctx, layers):
    labs = [seeded(100 + l, 64) for l in range(layers)]
    base, tree = fg.tree.ColumnTreeBuilder(ctx, layers, 8).add_final_columns(labs)
    g = GOLD[f"tree_c_{layers}x64"]
    assert rows_sha(base) == g["base_sha256"]
    assert ints(tree)[-1] == int(g["root"], 16)
    assert ints(tree) == P.tree_data(P.hash_columns(labs), 8, 0)


def test_tree_c_batched_uploads(ctx, tune):
    # ragged upload batches (100 columns each over 512 nodes) must not change the result
    labs = [seeded(200 + l, 512) for l in range(11)]
    ref_base = P.hash_columns(labs)
    tune.set("tree_batch", 100)
    base, tree = fg.tree.ColumnTreeBuilder(ctx, 11, 8).add_final_columns(labs)
    assert ints(base) == ref_base
    assert ints(tree) == P.tree_data(ref_base, 8, 0)


def test_tree_c_device_equals_host(ctx):
    nodes, layers = 512, 11
    labs = [seeded(300 + l, nodes) for l in range(layers)]
    b_host, t_host = fg.tree.ColumnTreeBuilder(ctx, layers, 8).add_final_columns(labs)
    flat = np.frombuffer(b"".join(fg.tree._fr_array(l).tobytes() for l in labs), dtype=np.uint8).copy()
    d_lab = torch.from_numpy(flat).cuda()
    d_base = torch.zeros(32 * nodes, dtype=torch.uint8, device="cuda")
    tsz = fg.tree.get_merkle_tree_cache_size(nodes, 8, 0)
    d_tree = torch.zeros(32 * tsz, dtype=torch.uint8, device="cuda")
    fg.tree.ColumnTreeBuilder(ctx, layers, 8).add_final_columns_dev(d_lab.data_ptr(), nodes, d_base.data_ptr(),
                                                                     d_tree.data_ptr())
    ctx.synchronize()
    assert d_base.cpu().numpy().tobytes() == b_host
    assert d_tree.cpu().numpy().tobytes() == t_host


@pytest.mark.parametrize("discard", [0, 2])
def test_tree_r_last(ctx, discard, tune):
    nodes = 512
    labels, data = seeded(11, nodes), seeded(12, nodes)
    data[0], labels[1] = P.R - 1, P.R - 1  # wrap-around in the encoding
    tune.set("tree_batch", 96)
    replica, tree = fg.tree.generate_tree_r_last(ctx, labels, data, 8, discard)
    ref_rep = [P.encode(k, d) for k, d in zip(labels, data)]
    assert ints(replica) == ref_rep
    assert ints(tree) == P.tree_data(ref_rep, 8, discard)


def test_tree_r_last_rejects_noncanonical_data(ctx):
    labels, data = seeded(13, 64), seeded(14, 64)
    data[5] = P.R + 3
    with pytest.raises(fg.FilGpuError):
        fg.tree.generate_tree_r_last(ctx, labels, data, 8, 0)


def test_large_tree_sampled_parents(ctx):
    # 8^7 = 2,097,152 leaves built on the device; 64 random parents (every level) re-hashed by the oracle
    n = 8 ** 7
    rng = np.random.default_rng(9)
    w = rng.integers(0, 2 ** 64, size=(n, 4), dtype=np.uint64)
    w[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)  # < 2^252 < r: canonical
    leaves = torch.from_numpy(w.view(np.uint8).reshape(-1)).cuda()
    tsz = fg.tree.get_merkle_tree_cache_size(n, 8, 0)
    tree = torch.zeros(32 * tsz, dtype=torch.uint8, device="cuda")
    from fil_groth16._lib import check, lib
    import ctypes
    check(lib().mi_tree_build_dev(ctx.h, 8, ctypes.c_void_p(leaves.data_ptr()), n, 0, ctypes.c_void_p(tree.data_ptr())))
    ctx.synchronize()
    rows = [w.view(np.uint8).reshape(-1)]
    t = tree.cpu().numpy()
    off, cnt = 0, n // 8
    while cnt >= 1:
        rows.append(t[32 * off:32 * (off + cnt)])
        off += cnt
        cnt //= 8
    h = P.poseidon(8)
    pr = random.Random(1)
    for level in range(1, len(rows)):
        for _ in range(8):
            j = pr.randrange(len(rows[level]) // 32)
            kids = [int.from_bytes(rows[level - 1][32 * (8 * j + q):32 * (8 * j + q + 1)].tobytes(), "little")
                    for q in range(8)]
            assert int.from_bytes(rows[level][32 * j:32 * (j + 1)].tobytes(), "little") == h.hash(kids), (level, j)


def test_large_tree_c_sampled_columns_and_parents(ctx):
    """BASELINE-scale property check: tree C over 2^24 columns x 11 layers (one 512 MiB-per-layer sub-tree,
    5.6 GB of labels in HBM); 256 random column hashes and every level's sampled parents are recomputed by
    the C oracle (or_poseidon_hash)."""
    import oracle_py

    n, L = 8 ** 8, 11
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    labels = torch.randint(0, 2 ** 62, (L * n, 4), dtype=torch.int64, device="cuda", generator=g)
    labels[:, 3] &= 0x0FFFFFFFFFFFFFFF
    base = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    tsz = fg.tree.get_merkle_tree_cache_size(n, 8, 0)
    tree = torch.zeros((tsz, 4), dtype=torch.int64, device="cuda")
    fg.tree.ColumnTreeBuilder(ctx, L, 8).add_final_columns_dev(labels.data_ptr(), n, base.data_ptr(), tree.data_ptr())
    ctx.synchronize()
    pr = random.Random(2)
    cols = sorted(pr.randrange(n) for _ in range(256))
    idx = torch.tensor(cols, device="cuda")
    lab = labels.view(L, n, 4)[:, idx].permute(1, 0, 2).contiguous().cpu().numpy().view(np.uint8).tobytes()
    want = oracle_py.poseidon_hash(11, lab)
    got = base[idx].cpu().numpy().view(np.uint8).tobytes()
    assert got == want
    t = tree.cpu().numpy().view(np.uint8).reshape(-1, 32)
    rows, off, cnt = [base.cpu().numpy().view(np.uint8).reshape(-1, 32)], 0, n // 8
    while cnt >= 1:
        rows.append(t[off:off + cnt])
        off += cnt
        cnt //= 8
    for level in range(1, len(rows)):
        js = [pr.randrange(len(rows[level])) for _ in range(16)]
        kids = b"".join(rows[level - 1][8 * j:8 * j + 8].tobytes() for j in js)
        assert oracle_py.poseidon_hash(8, kids) == b"".join(rows[level][j].tobytes() for j in js), level


def _proof_root(leaf, sibs, c, arity):
    """MerkleProof root from a leaf and its per-row siblings (position order, own slot = digit of c)."""
    h = P.poseidon(arity)
    cur = leaf
    for row in sibs:
        own = c % arity
        cur = h.hash(row[:own] + [cur] + row[own:])
        c //= arity
    return cur


@pytest.mark.parametrize("arity,n,discard", [(8, 512, 0), (8, 512, 1), (8, 4096, 2), (2, 256, 3), (4, 1024, 0)])
def test_inclusion_paths_vs_oracle(ctx, arity, n, discard):
    # gen_proof / gen_cached_proof (vanilla/proof.hpp:139-140,183-186): siblings equal the oracle tree's, and
    # every proof hashes back to the root; challenges cover both ends and repeats
    leaves = seeded(1000 + n + discard, n)
    rows = P.merkle_rows(leaves, arity)
    tree = fg.tree.TreeBuilder(ctx, arity, discard).add_final_leaves(leaves)
    d_leaves = torch.from_numpy(fg.tree._fr_array(leaves)).cuda()
    d_tree = torch.from_numpy(np.frombuffer(tree, dtype=np.uint8).copy()).cuda()
    chal = np.array([0, n - 1, 1, arity, n // 2, 5, 5] + list(np.random.default_rng(n).integers(0, n, 57)),
                    dtype=np.uint64)
    H = fg.tree.tree_height(n, arity)
    d_chal = torch.from_numpy(chal.view(np.int64)).cuda()
    d_leaf = torch.zeros(32 * len(chal), dtype=torch.uint8, device="cuda")
    d_sib = torch.zeros(32 * len(chal) * H * (arity - 1), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    fg.tree.gen_proofs_dev(ctx, arity, d_leaves.data_ptr(), n, discard, d_tree.data_ptr(), len(chal),
                           d_chal.data_ptr(), d_leaf.data_ptr(), d_sib.data_ptr())
    ctx.synchronize()
    got_leaf = ints(d_leaf.cpu().numpy())
    got_sib = ints(d_sib.cpu().numpy())
    root = rows[-1][0]
    for i, c in enumerate(int(x) for x in chal):
        assert got_leaf[i] == leaves[c]
        sibs = []
        for j in range(H):
            idx = c // arity ** j
            g = idx - idx % arity
            exp = [rows[j][g + s] for s in range(arity) if s != idx % arity]
            row = got_sib[(i * H + j) * (arity - 1):(i * H + j + 1) * (arity - 1)]
            assert row == exp, (c, j)
            sibs.append(row)
        assert _proof_root(got_leaf[i], sibs, c, arity) == root


def test_inclusion_paths_refuse_out_of_range(ctx):
    n = 64
    leaves = seeded(77, n)
    tree = fg.tree.TreeBuilder(ctx, 8, 0).add_final_leaves(leaves)
    d_leaves = torch.from_numpy(fg.tree._fr_array(leaves)).cuda()
    d_tree = torch.from_numpy(np.frombuffer(tree, dtype=np.uint8).copy()).cuda()
    d_chal = torch.tensor([3, n], dtype=torch.int64, device="cuda")
    d_leaf = torch.zeros(64, dtype=torch.uint8, device="cuda")
    d_sib = torch.zeros(32 * 2 * 2 * 7, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    with pytest.raises(fg.FilGpuError):
        fg.tree.gen_proofs_dev(ctx, 8, d_leaves.data_ptr(), n, 0, d_tree.data_ptr(), 2, d_chal.data_ptr(),
                               d_leaf.data_ptr(), d_sib.data_ptr())
    assert int(d_sib.sum()) == 0
