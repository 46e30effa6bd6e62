"""Deterministic test circuits (TEST INFRASTRUCTURE).

- toy_chain(n): BASELINE config 1 shape -- x_{i+1} = x_i^2 + k_i, public inputs [ONE, x_n].
- random_circuit(seed, ...): a satisfiable sparse R1CS exercising every density path of the
  bellman prover: inputs used in B (b_input_density), aux never in A (a_aux_density gaps), aux
  only in C, empty linear combinations (x * 0 = 0), repeated variables inside one LC and
  non-unit coefficients.

Variables: 0..n_in-1 are inputs (0 = ONE, the reference's convention,
porep/stacked/circuit/proof.cpp:120), then aux.
"""
import numpy as np

from pyref import R, SplitMix64, fr_le


def toy_chain(n_rows=1022, seed=1):
    rng = SplitMix64(seed)
    ks = [rng.next() % 1000 + 1 for _ in range(n_rows)]
    n_in, n_aux = 2, n_rows
    x = [3]
    for k in ks:
        x.append((x[-1] * x[-1] + k) % R)
    rows = []
    for j, k in enumerate(ks):
        xj = n_in + j
        nxt = 1 if j == n_rows - 1 else n_in + j + 1
        rows.append(([(xj, 1)], [(xj, 1)], [(nxt, 1), (0, (-k) % R)]))
    z = [1, x[n_rows]] + x[:n_rows]
    return n_in, n_aux, rows, z


def random_circuit(seed, n_rows, n_in=4, n_free=8):
    rng = SplitMix64(seed)
    z = [1] + [rng.fr() for _ in range(n_in - 1)] + [rng.fr() for _ in range(n_free)]
    rows = []

    def pick(nv):
        return rng.next() % nv

    def coeff():
        c = rng.next() % 5
        return 1 if c < 2 else (rng.fr() if c == 4 else (c + 1))

    for j in range(n_rows):
        nv = len(z)
        kind = rng.next() % 16
        if kind == 0:   # 0 * x = 0 with empty LCs
            rows.append(([(pick(nv), coeff())], [], []))
            continue
        A = [(pick(nv), coeff()) for _ in range(1 + rng.next() % 3)]
        if kind == 1:   # repeated variable inside one LC
            A.append((A[0][0], coeff()))
        B = [(pick(nv), coeff()) for _ in range(1 + rng.next() % 2)]
        if kind == 2:   # public input (not ONE) in B
            B.append((1 + rng.next() % (n_in - 1), coeff()))
        ev = lambda lc: sum(c * z[v] for v, c in lc) % R
        val = ev(A) * ev(B) % R
        C = [(len(z), 1)]
        if kind == 3:   # extra C term on ONE / an input
            v = rng.next() % n_in
            k = coeff()
            C.append((v, k))
            val = (val - k * z[v]) % R
        z.append(val)
        rows.append((A, B, C))
    n_aux = len(z) - n_in
    return n_in, n_aux, rows, z


def to_csr(rows):
    """-> list of 3 (row_ptr uint64[n+1], col uint32[nnz], coeff uint8[nnz*32])"""
    mats = []
    for m in range(3):
        rp = [0]
        cols, coeffs = [], []
        for row in rows:
            for v, c in row[m]:
                cols.append(v)
                coeffs.append(fr_le(c))
            rp.append(len(cols))
        mats.append((np.array(rp, dtype=np.uint64), np.array(cols, dtype=np.uint32),
                     np.frombuffer(b"".join(coeffs), dtype=np.uint8).copy()))
    return mats


def z_bytes(z):
    return b"".join(fr_le(v) for v in z)


TOXIC_SEED = 0x5EED


def toxic(seed=TOXIC_SEED):
    rng = SplitMix64(seed)
    return [rng.fr() for _ in range(5)]


def blinding(seed=1):
    rng = SplitMix64(seed)
    return rng.fr(), rng.fr()
