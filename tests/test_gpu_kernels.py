"""GPU parity: NTT and MSM kernels (through the C ABI) against the oracle and the golden vectors.

Bit-exact comparisons throughout (integer / field arithmetic).  Oracle = oracle/oracle.cpp,
itself pinned to tests/golden/golden.json (independent Python restatement + pairing check).
"""
import os
import random

import numpy as np
import pytest

import circuits
import fil_groth16 as fg
from pyref import R, SplitMix64

pytestmark = pytest.mark.gpu

KINDS = [(False, False), (True, False), (False, True), (True, True)]  # fft, ifft, coset_fft, icoset_fft


def rand_fr_bytes(n, seed):
    rng = np.random.default_rng(seed)
    words = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    words[:, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)  # < 2^254 < r
    return words.tobytes()


def test_ntt_golden(ctx, golden):
    for log_n, ent in golden["ntt"].items():
        inp = bytes.fromhex(ent["input"])
        for (inv, coset), name in zip(KINDS, ("fft", "ifft", "coset_fft", "icoset_fft")):
            assert ctx.ntt(inp, int(log_n), inv, coset).hex() == ent[name], (log_n, name)


@pytest.mark.parametrize("log_n", [0, 1, 2, 5, 9, 10, 11, 12, 13, 17, 18, 20])
def test_ntt_vs_oracle(ctx, oracle, log_n):
    data = rand_fr_bytes(1 << log_n, 100 + log_n)
    for kind, (inv, coset) in enumerate(KINDS):
        if log_n > 13 and kind in (1, 2):
            continue  # large sizes: fft + icoset cover both DIF passes with and without coset
        assert ctx.ntt(data, log_n, inv, coset) == oracle.ntt(data, log_n, kind), (log_n, kind)


def test_ntt_roundtrip_2_22(ctx):
    log_n = 22
    data = rand_fr_bytes(1 << log_n, 7)
    fwd = ctx.ntt(data, log_n, False, True)
    assert ctx.ntt(fwd, log_n, True, True) == data


def test_ntt_non_canonical_input_reduced(ctx, oracle):
    # inputs >= r are reduced mod r at the boundary (2^256 - 1 -> 2^256 - 1 - 2r)
    vals = [R + 5, 2**256 - 1, 3, R - 1]
    data = b"".join(v.to_bytes(32, "little") for v in vals)
    red = b"".join((v % R).to_bytes(32, "little") for v in vals)
    assert ctx.ntt(data, 2, False, False) == oracle.ntt(red, 2, 0)


def test_msm_golden(ctx, golden):
    g1 = golden["msm"]["g1"]
    assert ctx.msm_g1(bytes.fromhex(g1["bases"]), bytes.fromhex(g1["scalars"])).hex() == g1["result"]
    g2 = golden["msm"]["g2"]
    assert ctx.msm_g2(bytes.fromhex(g2["bases"]), bytes.fromhex(g2["scalars"])).hex() == g2["result"]


def _bases_g1(oracle, n, seed):
    rng = SplitMix64(seed)
    return oracle.g1_fixed_base([rng.fr() for _ in range(n)])


def _bases_g2(oracle, n, seed):
    rng = SplitMix64(seed)
    return oracle.g2_fixed_base([rng.fr() for _ in range(n)])


@pytest.mark.parametrize("n", [1, 2, 3, 31, 64, 257, 1000, 4096, 20000])
def test_msm_g1_random(ctx, oracle, n):
    bases = _bases_g1(oracle, n, 1000 + n)
    scal = rand_fr_bytes(n, 2000 + n)
    assert ctx.msm_g1(bases, scal) == oracle.msm_g1(bases, scal)


@pytest.fixture(params=["0", "2"])
def g2_level2(request, tune):
    """G2 bucket reduction: "0" the running-sum kernels, "2" the second-level MSM over affine buckets
    (forced at every size; by default it takes over from 2^20 level-1 buckets, g2_l2)."""
    tune.set("g2_l2", int(request.param))
    return request.param


@pytest.mark.parametrize("n", [1, 5, 100, 1500])
def test_msm_g2_random(ctx, oracle, n, g2_level2):
    bases = _bases_g2(oracle, n, 3000 + n)
    scal = rand_fr_bytes(n, 4000 + n)
    assert ctx.msm_g2(bases, scal) == oracle.msm_g2(bases, scal)


def test_msm_edge_scalars(ctx, oracle):
    n = 3000
    bases = _bases_g1(oracle, n, 77)
    zeros = bytes(32 * n)
    assert ctx.msm_g1(bases, zeros) == oracle.msm_g1(bases, zeros)  # identity
    ones = (1).to_bytes(32, "little") * n  # every entry in one bucket (boolean witnesses)
    assert ctx.msm_g1(bases, ones) == oracle.msm_g1(bases, ones)
    mx = (R - 1).to_bytes(32, "little") * n
    assert ctx.msm_g1(bases, mx) == oracle.msm_g1(bases, mx)
    # mixture of 0/1/small and a repeated base (P + P hits the doubling branch)
    rng = random.Random(5)
    sc = [rng.choice([0, 1, 1, 2, 3, R - 1, rng.randrange(R)]) for _ in range(n)]
    sb = b"".join(s.to_bytes(32, "little") for s in sc)
    rep = bases[:96] * n
    assert ctx.msm_g1(rep, sb) == oracle.msm_g1(rep, sb)
    assert ctx.msm_g1(bases, sb) == oracle.msm_g1(bases, sb)
    # P and -P together: bucket sum hits the P + (-P) = O branch
    g = oracle.g1_generator()
    neg = oracle.g1_mul(g, R - 1)
    pts = (g + neg) * 8
    one = (1).to_bytes(32, "little") * 16
    assert ctx.msm_g1(pts, one) == oracle.msm_g1(pts, one)


def test_msm_infinity_bases(ctx, oracle):
    n = 50
    bases = bytearray(_bases_g1(oracle, n, 9))
    for i in (0, 7, 49):
        bases[96 * i:96 * i + 96] = bytes([0x40]) + bytes(95)
    scal = rand_fr_bytes(n, 10)
    assert ctx.msm_g1(bytes(bases), scal) == oracle.msm_g1(bytes(bases), scal)


def test_msm_rejects_bad_points(ctx, oracle):
    bases = bytearray(_bases_g1(oracle, 4, 11))
    bases[100] ^= 0x01  # corrupt x of point 1 -> off curve
    with pytest.raises(fg.FilGpuError):
        ctx.msm_g1(bytes(bases), rand_fr_bytes(4, 12))


@pytest.fixture(params=["auto", "windowed"])
def sort_mode(request, tune):
    """auto: 2^20 sorts every window in one call; windowed: the per-window sort with zero-digit
    compaction that MSMs of 2^22+ points take (msm_sort, read at every MSM)."""
    tune.set("msm_sort", 1 if request.param == "windowed" else 0)
    return request.param


def test_msm_g1_linearity_2_20(ctx, oracle, sort_mode):
    """Size-independent check at the BASELINE config-2 size: bases k_i G with known k_i, so
    MSM(bases, s) == (sum s_i k_i) G.  The Fr dot product is computed in Python ints."""
    n = 1 << 20
    rng = np.random.default_rng(42)
    kw = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    kw[:, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)
    kb = kw.tobytes()
    bases = oracle.g1_fixed_base(kb)
    sb = rand_fr_bytes(n, 43)
    got = ctx.msm_g1(bases, sb)
    k = np.frombuffer(kb, dtype=np.uint64).reshape(n, 4)
    s = np.frombuffer(sb, dtype=np.uint64).reshape(n, 4)
    acc = 0
    for i in range(0, n, 4096):  # python ints, chunked
        kk = [int(a) | int(b) << 64 | int(c) << 128 | int(d) << 192 for a, b, c, d in k[i:i + 4096]]
        ss = [int(a) | int(b) << 64 | int(c) << 128 | int(d) << 192 for a, b, c, d in s[i:i + 4096]]
        acc = (acc + sum(x * y for x, y in zip(kk, ss))) % R
    assert got == oracle.g1_mul(oracle.g1_generator(), acc)


def test_msm_g1_boolean_heavy_2_20(ctx, oracle, sort_mode):
    """Boolean-heavy scalars (Filecoin witnesses): ~2^19 entries land in bucket 1 of window 0, so
    the in-place chunk tree runs four levels.  Checked by linearity on bases k_i G."""
    n = 1 << 20
    rng = np.random.default_rng(7)
    kw = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    kw[:, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)
    kb = kw.tobytes()
    bases = oracle.g1_fixed_base(kb)
    sel = rng.integers(0, 16, size=n)
    sw = np.zeros((n, 4), dtype=np.uint64)
    sw[sel < 9, 0] = 1  # ~56% ones, ~6% random, rest zero
    rnd = sel == 15
    sw[rnd] = rng.integers(0, 2**64, size=(int(rnd.sum()), 4), dtype=np.uint64)
    sw[rnd, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
    sb = sw.tobytes()
    got = ctx.msm_g1(bases, sb)
    acc = 0
    for i in range(0, n, 4096):
        kk = [int(a) | int(b) << 64 | int(c) << 128 | int(d) << 192 for a, b, c, d in kw[i:i + 4096]]
        ss = [int(a) | int(b) << 64 | int(c) << 128 | int(d) << 192 for a, b, c, d in sw[i:i + 4096]]
        acc = (acc + sum(x * y for x, y in zip(kk, ss))) % R
    assert got == oracle.g1_mul(oracle.g1_generator(), acc)


def test_msm_g2_boolean_heavy(ctx, oracle, sort_mode, g2_level2):
    """G2 with one huge bucket (three tree levels) next to random scalars, against the oracle."""
    n = 1 << 16
    bases = _bases_g2(oracle, n, 555)
    rng = random.Random(556)
    sc = [1 if rng.random() < 0.8 else rng.randrange(R) for _ in range(n)]
    sb = b"".join(s.to_bytes(32, "little") for s in sc)
    assert ctx.msm_g2(bases, sb) == oracle.msm_g2(bases, sb)


def _split_scalars(n, seed):
    """full-width, zero, one, R - 1, 128-bit-only (empty high half) and high-half-only scalars"""
    rng = np.random.default_rng(seed)
    w = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    w[:, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)
    kind = rng.integers(0, 8, size=n)
    w[kind == 1] = 0
    w[kind == 2] = np.array([1, 0, 0, 0], dtype=np.uint64)
    w[kind == 3] = np.frombuffer((R - 1).to_bytes(32, "little"), dtype=np.uint64)
    w[kind == 4, 2:] = 0
    w[kind == 5, :2] = 0
    return w.tobytes()


@pytest.mark.parametrize("split", ["0", "2", "glv"])
def test_msm_split_tables_vs_oracle(ctx, oracle, tune, split):
    """Split mode (msm_split=2 forces it at any size): the l and a queries' MSMs over their 2^128
    tables, against the oracle's MSM over the same points; "glv": keys generated and MSMs run with
    msm_glv=1 (no tables)."""
    import torch

    tune.set("msm_split", int("2" if split == "glv" else split))
    tune.set("msm_glv", int("1" if split == "glv" else "0"))
    tune.set("msm_wt_max_log", 0)  # split / plain paths, not the key's window tables
    n_in, n_aux, rws, z = circuits.random_circuit(91, 3000, n_in=6, n_free=32)
    gc = fg.Circuit(ctx, len(rws), n_in, n_aux, circuits.to_csr(rws))
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    for which in (1, 2):
        pts, q = pk.points(which), pk.query(which)
        n = len(q) // 96
        for seed in (1, 2):
            sb = _split_scalars(n, 100 * which + seed)
            sd = torch.from_numpy(np.frombuffer(sb, dtype=np.uint8).copy()).cuda()
            assert pts.msm_dev(sd.data_ptr(), n) == oracle.msm_g1(q, sb), (which, seed)
            torch.cuda.synchronize()


def test_msm_split_default_2_17(ctx, oracle, tune):
    """Default selection (split from 2^16 points on) on the l query of a 2^17-row synthetic circuit."""
    import torch

    tune.set("msm_wt_max_log", 0)  # the split path, not the key's window tables
    from fil_groth16 import synth

    sc = synth.SynthCircuit(log_rows=17, n_in=4, seed=3)
    gc = sc.load(ctx)
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    pts, q = pk.points(1), pk.query(1)
    n = len(q) // 96
    assert n >= 1 << 16
    sb = _split_scalars(n, 5)
    sd = torch.from_numpy(np.frombuffer(sb, dtype=np.uint8).copy()).cuda()
    assert pts.msm_dev(sd.data_ptr(), n) == oracle.msm_g1(q, sb)


GLV_LAMBDA = 0xAC45A4010001A40200000000FFFFFFFF  # csrc/glv.h: phi(P) = lambda P, lambda^2 + lambda + 1 = r


def _glv_scalars(n, seed):
    """random, zero, one and the decomposition's edges: lambda - 1, lambda, lambda + 1, 2^128 +- 1,
    r - 1 = lambda^2 + lambda, lambda^2, r - lambda"""
    rng = random.Random(seed)
    edges = [0, 1, GLV_LAMBDA - 1, GLV_LAMBDA, GLV_LAMBDA + 1, 2**128 - 1, 2**128, 2**128 + 1, R - 1,
             GLV_LAMBDA**2 % R, R - GLV_LAMBDA, 2]
    sc = [edges[i] if i < len(edges) else rng.choice([rng.randrange(R), rng.randrange(2**128), 0, 1,
                                                       rng.choice(edges)]) for i in range(n)]
    return b"".join(x.to_bytes(32, "little") for x in sc)


@pytest.mark.parametrize("n,c", [(1, ""), (13, ""), (5000, ""), (5000, "12"), (5000, "22")])
def test_msm_glv_vs_oracle(ctx, oracle, tune, n, c):
    """G1 split mode through the GLV endomorphism (msm_glv=1; msm_split=2 forces split at any size)
    over caller-uploaded bases, which have no 2^128 table: edge scalars of the k = k1 + lambda k2
    decomposition, at the default window, c = 12 and the production c = 22 (2^22 sub-buckets per window)."""
    tune.set("msm_glv", 1)
    tune.set("msm_split", 2)
    if c:
        tune.set("msm_c", int(c))
    bases = _bases_g1(oracle, n, 555 + n)
    sb = _glv_scalars(n, 7 + n)
    assert ctx.msm_g1(bases, sb) == oracle.msm_g1(bases, sb)


def test_msm_glv_repeated_base_and_negation(ctx, oracle, tune):
    """GLV sub-bucket merge branches: one base repeated (P and phi(P) sums in the same bucket), P with -P
    (a sub-bucket sum at infinity), and scalars lambda / 1 on the same base (phi(P) + ... hits the doubling
    of the merge when k2 = 1, k1 = 0 meets k1 = 1)."""
    tune.set("msm_glv", 1)
    tune.set("msm_split", 2)
    g = oracle.g1_generator()
    neg = oracle.g1_mul(g, R - 1)
    pts = (g + neg) * 20 + g * 24
    rng = random.Random(3)
    sc = [GLV_LAMBDA, 1, 1, GLV_LAMBDA] * 16
    sc = [rng.choice(sc + [rng.randrange(R)]) for _ in range(len(pts) // 96)]
    sb = b"".join(x.to_bytes(32, "little") for x in sc)
    assert ctx.msm_g1(pts, sb) == oracle.msm_g1(pts, sb)
    lam_pts = g * 8
    lam_sc = b"".join(x.to_bytes(32, "little") for x in [GLV_LAMBDA, 1, GLV_LAMBDA + 1, 0, GLV_LAMBDA, 1, 2, 3])
    assert ctx.msm_g1(lam_pts, lam_sc) == oracle.msm_g1(lam_pts, lam_sc)


def test_msm_glv_boolean_heavy_2_20(ctx, oracle, tune):
    """GLV at the 2^20 config-2 size with Filecoin-like boolean-heavy scalars, against the table-free
    plain path's result (the plain path is pinned against the oracle by the linearity tests)."""
    tune.set("msm_split", 2)
    n = 1 << 20
    rng = np.random.default_rng(11)
    small = _bases_g1(oracle, 64, 91)
    bases = small * (n // 64)
    kind = rng.integers(0, 10, size=n)
    w = np.zeros((n, 4), dtype=np.uint64)
    w[kind < 6, 0] = 1
    w[kind == 6, 0] = rng.integers(2, 2**20, size=int((kind == 6).sum()), dtype=np.uint64)
    full = kind >= 8
    w[full] = rng.integers(0, 2**64, size=(int(full.sum()), 4), dtype=np.uint64)
    w[full, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)
    sb = w.tobytes()
    tune.set("msm_glv", 0)
    tune.set("msm_split", 0)
    plain = ctx.msm_g1(bases, sb)
    tune.set("msm_glv", 1)
    tune.set("msm_split", 2)
    assert ctx.msm_g1(bases, sb) == plain
    # and the oracle on the 64 distinct bases: sum over i of s_i P_(i mod 64) = sum_j (sum_{i = j mod 64} s_i) P_j
    agg = [0] * 64
    ints = [int.from_bytes(sb[32 * i:32 * i + 32], "little") for i in range(n)]
    for i, v in enumerate(ints):
        agg[i % 64] = (agg[i % 64] + v) % R
    ab = b"".join(x.to_bytes(32, "little") for x in agg)
    assert plain == oracle.msm_g1(small, ab)


def test_msm_glv_auto_uploaded_bases(ctx, oracle, tune):
    """Default policy (msm_glv unset): caller-uploaded bases have no 2^128 table, so a split-size G1 MSM
    takes the GLV split; the same MSM with msm_glv=0 runs the plain 256-bit path."""
    tune.clear("msm_glv")
    tune.set("msm_split", 2)
    n = 3001
    bases = _bases_g1(oracle, n, 4242)
    sb = _glv_scalars(n, 99)
    want = oracle.msm_g1(bases, sb)
    assert ctx.msm_g1(bases, sb) == want
    tune.set("msm_glv", 0)
    assert ctx.msm_g1(bases, sb) == want


# ---- fixed-base window tables (mi_points_precompute; small keys build them at load) ----

@pytest.mark.parametrize("n,c", [(1, 8), (3, 13), (1000, 8), (1000, 16), (20000, 13), (20000, 20)])
def test_msm_window_table_vs_oracle(ctx, oracle, n, c):
    """Every window's digits in one bucket set over T[w n + i] = 2^(c w) P_i: the same sum as the oracle's MSM, for
    uniform, zero, one, r - 1 and half-width scalars; prefixes of the table (MSMs over fewer points than it holds)
    too.  c = 8 and 20 bracket the window sizes (32 / 13 windows, 128 / 2^19 buckets)."""
    import torch

    bases = _bases_g1(oracle, n, 5000 + n)
    pts = fg.Points(ctx, bases)
    pts.precompute(c)
    assert pts.table_info() == {"window_bits": c, "windows": -(-256 // c), "points": n}
    ctx.reset_stats()
    for seed in (1, 2):
        sb = _split_scalars(n, 10 * n + seed)
        sd = torch.from_numpy(np.frombuffer(sb, dtype=np.uint8).copy()).cuda()
        assert pts.msm_dev(sd.data_ptr(), n) == oracle.msm_g1(bases, sb), (n, c, seed)
        m = max(1, n // 3)
        assert pts.msm_dev(sd.data_ptr(), m) == oracle.msm_g1(bases[:96 * m], sb[:32 * m]), (n, c, seed, m)
    assert ctx.table_msms() == 4


@pytest.mark.parametrize("bitsum", ["1", "0"])
def test_msm_window_table_linearity_2_20(ctx, oracle, tune, bitsum):
    """BASELINE config-2 size over a window table at the library's window choice and at c = 20 (2^19 buckets in
    one window): MSM(k_i G, s_i) == (sum s_i k_i) G.  bitsum "0" reduces the one window with the running-sum
    kernels instead of the bit-row sums (msm_bitsum)."""
    import torch

    tune.set("msm_bitsum", int(bitsum))
    n = 1 << 20
    rng = np.random.default_rng(420)
    kw = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    kw[:, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)
    kb = kw.tobytes()
    pts = fg.Points(ctx, oracle.g1_fixed_base(kb))
    sb = rand_fr_bytes(n, 421)
    s = np.frombuffer(sb, dtype=np.uint64).reshape(n, 4)
    acc = 0
    for i in range(0, n, 4096):
        kk = [int(a) | int(b) << 64 | int(c) << 128 | int(d) << 192 for a, b, c, d in kw[i:i + 4096]]
        ss = [int(a) | int(b) << 64 | int(c) << 128 | int(d) << 192 for a, b, c, d in s[i:i + 4096]]
        acc = (acc + sum(x * y for x, y in zip(kk, ss))) % R
    want = oracle.g1_mul(oracle.g1_generator(), acc)
    sd = torch.from_numpy(np.frombuffer(sb, dtype=np.uint8).copy()).cuda()
    for c in (0, 20):
        pts.precompute(c)
        assert pts.msm_dev(sd.data_ptr(), n) == want, (c, pts.table_info())


def test_msm_window_table_boolean_heavy(ctx, oracle):
    """Boolean-heavy scalars over a table: every window-0 digit 1 lands in one bucket (a deep chunk tree),
    the other windows' digits are zero."""
    import torch

    n = 1 << 16
    bases = _bases_g1(oracle, n, 6001)
    rng = random.Random(6002)
    sc = [1 if rng.random() < 0.7 else (0 if rng.random() < 0.5 else rng.randrange(R)) for _ in range(n)]
    sb = b"".join(v.to_bytes(32, "little") for v in sc)
    pts = fg.Points(ctx, bases)
    pts.precompute(16)
    sd = torch.from_numpy(np.frombuffer(sb, dtype=np.uint8).copy()).cuda()
    assert pts.msm_dev(sd.data_ptr(), n) == oracle.msm_g1(bases, sb)


@pytest.mark.parametrize("n,c", [(1, 8), (700, 13), (5000, 16)])
def test_msm_g2_window_table_vs_oracle(ctx, oracle, n, c):
    """G2 bases over a window table (lane-pair accumulation and bit-row reduction) against the oracle."""
    import torch

    bases = _bases_g2(oracle, n, 7000 + n)
    pts = fg.Points(ctx, bases, g2=True)
    pts.precompute(c)
    assert pts.table_info() == {"window_bits": c, "windows": -(-256 // c), "points": n}
    ctx.reset_stats()
    sb = _split_scalars(n, 7100 + n)
    sd = torch.from_numpy(np.frombuffer(sb, dtype=np.uint8).copy()).cuda()
    assert pts.msm_dev(sd.data_ptr(), n) == oracle.msm_g2(bases, sb), (n, c)
    assert ctx.table_msms(g2=True) == 1 and ctx.table_msms() == 0


def test_precompute_argument_rules(ctx, oracle):
    bases = _bases_g1(oracle, 16, 6003)
    pts = fg.Points(ctx, bases)
    for bad in ((7, 16), (23, 16), (16, 0), (16, 17)):
        with pytest.raises(fg.FilGpuError):
            pts.precompute(*bad)
    assert pts.table_info() == {"window_bits": 0, "windows": 0, "points": 0}
    pts.precompute(16, 8)
    assert pts.table_info()["points"] == 8
