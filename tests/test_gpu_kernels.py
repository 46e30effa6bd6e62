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
def g2_level2(request, monkeypatch):
    """G2 bucket reduction: "0" the running-sum kernels, "2" the second-level MSM over affine buckets
    (forced at every size; by default it takes over from 2^20 level-1 buckets, MI_G2_L2)."""
    monkeypatch.setenv("MI_G2_L2", request.param)
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
def sort_mode(request, monkeypatch):
    """auto: 2^20 sorts every window in one call; windowed: the per-window sort with zero-digit
    compaction that MSMs of 2^22+ points take (MI_MSM_SORT, read at every MSM)."""
    monkeypatch.setenv("MI_MSM_SORT", request.param)
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


@pytest.mark.parametrize("split", ["0", "2"])
def test_msm_split_tables_vs_oracle(ctx, oracle, monkeypatch, split):
    """Split mode (MI_MSM_SPLIT=2 forces it at any size): the l and a queries' MSMs over their 2^128
    tables, against the oracle's MSM over the same points."""
    import torch

    monkeypatch.setenv("MI_MSM_SPLIT", split)
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


def test_msm_split_default_2_17(ctx, oracle):
    """Default selection (split from 2^16 points on) on the l query of a 2^17-row synthetic circuit."""
    import torch

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
