"""GPU parity: SDR labelling witness through the C ABI -- k_sdr_labels (parents per
entry, the LabelingProof form) and k_sdr_labels_gather (parents gathered from device-resident layers, the
prove_layers loop of vanilla/proof.hpp:190-255) -- bit-exact against the oracle (oracle.cpp or_sdr_labels)
and tests/golden/sdr_golden.json (hashlib-generated).  SHA-256 is pinned by FIPS vectors in
tests/test_cpu_sdr.py; the message layout is parity unpinned (no reference label vector)."""
import json
import os

import numpy as np
import pytest
import torch

import fil_groth16 as fg

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "sdr_golden.json")))


def test_sdr_golden(ctx):
    for c in GOLD["cases"]:
        par = b"".join(bytes.fromhex(p) for p in c["parents"])
        got = fg.sdr.create_labels(ctx, bytes.fromhex(c["replica_id"]), [c["layer"]], [c["node"]], par,
                                   len(c["parents"]))
        assert got.hex() == c["label"], c


@pytest.mark.parametrize("n,n_parents", [(1, 37), (63, 14), (257, 6), (1000, 37), (4099, 14), (20000, 1),
                                         (300, 0)])
def test_sdr_labels_vs_oracle(ctx, oracle, n, n_parents):
    rng = np.random.default_rng(n * 41 + n_parents)
    rid = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    layers = rng.integers(1, 12, n, dtype=np.uint32)
    nodes = rng.integers(0, 2 ** 62, n, dtype=np.uint64)
    par = rng.integers(0, 256, 32 * n_parents * n, dtype=np.uint8).tobytes()
    got = fg.sdr.create_labels(ctx, rid, layers, nodes, par, n_parents)
    assert got == oracle.sdr_labels(rid, layers, nodes, par, n_parents)


def test_sdr_labeling_proof_objects(ctx, oracle):
    rng = np.random.default_rng(7)
    rid = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    ps = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(14)]
    lp = fg.sdr.LabelingProof(fg.sdr.repeat_parents(ps), 4, 123456)
    lab = lp.create_label(ctx, rid)
    assert lab == oracle.sdr_labels(rid, [4], [123456], b"".join(ps), 14)
    assert lp.verify(ctx, rid, lab) and not lp.verify(ctx, rid, bytes(32))
    data = (5).to_bytes(32, "little")
    ep = fg.sdr.EncodingProof(lp.parents, 4, 123456)
    assert ep.verify(ctx, rid, fg.sdr.encode(lab, data), data)
    assert not ep.verify(ctx, rid, fg.sdr.encode(lab, (6).to_bytes(32, "little")), data)


def test_sdr_empty_and_bad_arguments(ctx):
    rid = bytes(32)
    assert fg.sdr.create_labels(ctx, rid, [], [], b"", 14) == b""
    with pytest.raises(fg.FilGpuError):
        fg.sdr.create_labels(ctx, rid, [1], [1], bytes(32 * 38), 38)


def _layers_setup(n_layers, nodes, count, seed):
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, 256, (n_layers, nodes, 32), dtype=np.uint8)
    layers = rng.integers(1, n_layers + 1, count, dtype=np.uint32)
    chal = rng.integers(1, nodes, count, dtype=np.uint64)
    pidx = rng.integers(0, nodes, (count, 14), dtype=np.uint32)
    return rng, labels, layers, chal, pidx


def _host_parents(labels, layer, pidx_row):
    # vanilla/proof.hpp:196-231: layer 1 -> the 6 base parents of layer 1; else 6 base parents of the layer
    # and 8 expander parents of the layer below
    if layer == 1:
        return [labels[0, p].tobytes() for p in pidx_row[:6]]
    return [labels[layer - 1, p].tobytes() for p in pidx_row[:6]] + \
           [labels[layer - 2, p].tobytes() for p in pidx_row[6:]]


@pytest.mark.parametrize("prefetch", ["0", "1"])
@pytest.mark.parametrize("n_layers,nodes,count", [(2, 64, 50), (11, 4096, 3000)])
def test_sdr_labeling_proofs_gather_vs_oracle(ctx, oracle, n_layers, nodes, count, prefetch, tune):
    tune.set("sdr_prefetch", int(prefetch))  # both gather forms (software-pipelined or not)
    rng, labels, layers, chal, pidx = _layers_setup(n_layers, nodes, count, nodes + count)
    rid = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    dev = torch.device("cuda:0")
    L = torch.from_numpy(labels.reshape(-1)).to(dev)
    ly = torch.from_numpy(layers.view(np.int32)).to(dev)
    ch = torch.from_numpy(chal.view(np.int64)).to(dev)
    pi = torch.from_numpy(pidx.view(np.int32)).to(dev)
    out = torch.empty(count * 32, dtype=torch.uint8, device=dev)
    full = torch.empty(count * 37 * 32, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    fg.sdr.labeling_proofs_dev(ctx, rid, n_layers, nodes, L.data_ptr(), count, ly.data_ptr(), ch.data_ptr(),
                               pi.data_ptr(), out.data_ptr(), full.data_ptr())
    ctx.synchronize()
    got = out.cpu().numpy().tobytes()
    got_full = full.cpu().numpy().tobytes()
    exp = bytearray()
    exp_full = bytearray()
    for i in range(count):
        ps = _host_parents(labels, int(layers[i]), pidx[i])
        exp += oracle.sdr_labels(rid, [int(layers[i])], [int(chal[i])], b"".join(ps), len(ps))
        exp_full += b"".join(fg.sdr.repeat_parents(ps))
    assert got == bytes(exp)
    assert got_full == bytes(exp_full)


def test_sdr_labeling_proofs_refuse_out_of_range(ctx):
    n_layers, nodes, count = 3, 128, 40
    rng, labels, layers, chal, pidx = _layers_setup(n_layers, nodes, count, 9)
    dev = torch.device("cuda:0")
    L = torch.from_numpy(labels.reshape(-1)).to(dev)
    ch = torch.from_numpy(chal.view(np.int64)).to(dev)
    out = torch.zeros(count * 32, dtype=torch.uint8, device=dev)
    bad_idx = pidx.copy()
    bad_idx[17, 9] = nodes  # one expander parent past the layer
    bad_layers = layers.copy()
    bad_layers[3] = n_layers + 1
    for ly_np, pi_np in ((layers, bad_idx), (bad_layers, pidx)):
        ly = torch.from_numpy(ly_np.view(np.int32)).to(dev)
        pi = torch.from_numpy(pi_np.view(np.int32)).to(dev)
        torch.cuda.synchronize()
        with pytest.raises(fg.FilGpuError):
            fg.sdr.labeling_proofs_dev(ctx, bytes(32), n_layers, nodes, L.data_ptr(), count, ly.data_ptr(),
                                       ch.data_ptr(), pi.data_ptr(), out.data_ptr())
    assert int(out.sum()) == 0  # nothing was written


def test_sdr_labels_dev_large_sampled(ctx, oracle):
    # 2^20 labels with 14 parents each on the device; a seeded sample of 2048 checked against the oracle
    n, np_ = 1 << 20, 14
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    par = torch.randint(0, 256, (n * np_ * 32,), dtype=torch.uint8, device=dev, generator=g)
    layers = torch.randint(1, 12, (n,), dtype=torch.int32, device=dev, generator=g)
    nodes = torch.randint(0, 2 ** 40, (n,), dtype=torch.int64, device=dev, generator=g)
    out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    rid = bytes(range(32))
    torch.cuda.synchronize()
    fg.sdr.create_labels_dev(ctx, rid, n, layers.data_ptr(), nodes.data_ptr(), par.data_ptr(), np_, out.data_ptr())
    ctx.synchronize()
    idx = np.random.default_rng(5).choice(n, 2048, replace=False)
    idx_t = torch.from_numpy(idx).to(dev)
    s_par = par.view(n, np_ * 32)[idx_t].cpu().numpy().tobytes()
    s_lay = layers[idx_t].cpu().numpy().astype(np.uint32)
    s_nod = nodes[idx_t].cpu().numpy().astype(np.uint64)
    got = out.view(n, 32)[idx_t].cpu().numpy().tobytes()
    assert got == oracle.sdr_labels(rid, s_lay, s_nod, s_par, np_)


def _tree_d_rows(leaves):
    import hashlib

    rows = [leaves]
    while len(rows[-1]) > 1:
        cur = rows[-1]
        nxt = []
        for i in range(0, len(cur), 2):
            d = bytearray(hashlib.sha256(cur[i] + cur[i + 1]).digest())
            d[31] &= 0x3F
            nxt.append(bytes(d))
        rows.append(nxt)
    return rows


@pytest.mark.parametrize("n", [2, 1024])
def test_tree_d_vs_hashlib_and_openings(ctx, n):
    # tree D rows against a hashlib build of the same binary tree; openings through the shared path kernel
    rng = np.random.default_rng(n)
    raw = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    raw[:, 31] &= 0x3F  # Fr32-padded data nodes
    leaves = [raw[i].tobytes() for i in range(n)]
    rows = _tree_d_rows(leaves)
    dev = torch.device("cuda:0")
    d_leaves = torch.from_numpy(raw.reshape(-1).copy()).to(dev)
    d_tree = torch.zeros((n - 1) * 32, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    fg.sdr.build_tree_d_dev(ctx, d_leaves.data_ptr(), n, d_tree.data_ptr())
    ctx.synchronize()
    assert d_tree.cpu().numpy().tobytes() == b"".join(b"".join(r) for r in rows[1:])
    chal = np.array([0, n - 1, n // 3], dtype=np.uint64)
    H = fg.tree.tree_height(n, 2)
    d_chal = torch.from_numpy(chal.view(np.int64)).to(dev)
    d_leaf = torch.zeros(32 * 3, dtype=torch.uint8, device=dev)
    d_sib = torch.zeros(32 * 3 * H, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    fg.sdr.tree_d_proofs_dev(ctx, d_leaves.data_ptr(), n, d_tree.data_ptr(), 3, d_chal.data_ptr(),
                             d_leaf.data_ptr(), d_sib.data_ptr())
    ctx.synchronize()
    sib = d_sib.cpu().numpy().tobytes()
    for i, c in enumerate(int(x) for x in chal):
        assert d_leaf.cpu().numpy().tobytes()[32 * i:32 * i + 32] == leaves[c]
        for j in range(H):
            idx = c >> j
            assert sib[32 * (i * H + j):32 * (i * H + j + 1)] == rows[j][idx ^ 1], (c, j)


def test_tree_d_refuses_bad_shape(ctx):
    with pytest.raises(fg.FilGpuError):
        fg.sdr.build_tree_d_dev(ctx, 1, 3, 1)  # not a power of two: refused before any launch


@pytest.mark.parametrize("leaves", [4, 64])
def test_tree_d_root_matches_reference_comm_d(ctx, leaves):
    """mi_tree_d_build_dev over an empty 128-byte / 2048-byte sector: the root must equal the reference's
    compute_comm_d vectors (libs/filecoin/test/pieces.cpp:86-95). This pins the SHA-256 node hash and
    the byte-31 truncation that the label kernel shares."""
    from test_cpu_sdr import COMM_D_EMPTY

    dev = torch.device("cuda:0")
    d_leaves = torch.zeros(leaves * 32, dtype=torch.uint8, device=dev)
    d_tree = torch.zeros((leaves - 1) * 32, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    fg.sdr.build_tree_d_dev(ctx, d_leaves.data_ptr(), leaves, d_tree.data_ptr())
    ctx.synchronize()
    assert d_tree.cpu().numpy().tobytes()[-32:] == COMM_D_EMPTY[leaves]
