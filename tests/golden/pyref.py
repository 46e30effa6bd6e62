"""Independent pure-Python restatement of BLS12-381 / bellman Groth16 (TEST INFRASTRUCTURE).

Written separately from oracle/oracle.cpp (affine/Jacobian over Python ints, recursive-free
iterative FFT, naive multiexp, py_ecc-style pairing) so that agreement between the two is
evidence, not tautology.  Used only by tests/golden/gen_golden.py to produce the committed
fixtures and by a few slow CPU tests.

Reference anchors (crypto3 hot path is [NOT IN TREE]):
  - params layout scheme_params{vk,h,l,a,b_g1,b_g2}: core/crypto/scheme_params.hpp:46-66
  - density rule ("polynomials that evaluate to zero are omitted"): mapped_scheme_params.hpp:72-81
  - input ordering ONE first: porep/stacked/circuit/proof.cpp:120 (test), proof.hpp:186-269
  - 192-byte proof: proofs/constants.hpp:93
"""

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001

G1X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1
G2X = (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
       0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E)
G2Y = (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
       0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE)


# ----------------------------------------------------------------------------- fields
class Fq:
    zero = 0
    one = 1

    @staticmethod
    def add(a, b): return (a + b) % P

    @staticmethod
    def sub(a, b): return (a - b) % P

    @staticmethod
    def mul(a, b): return (a * b) % P

    @staticmethod
    def neg(a): return (-a) % P

    @staticmethod
    def inv(a): return pow(a, P - 2, P)

    @staticmethod
    def is_zero(a): return a == 0


class Fq2:
    zero = (0, 0)
    one = (1, 0)

    @staticmethod
    def add(a, b): return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)

    @staticmethod
    def sub(a, b): return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)

    @staticmethod
    def mul(a, b):
        return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)

    @staticmethod
    def neg(a): return ((-a[0]) % P, (-a[1]) % P)

    @staticmethod
    def inv(a):
        n = pow((a[0] * a[0] + a[1] * a[1]) % P, P - 2, P)
        return ((a[0] * n) % P, (-a[1] * n) % P)

    @staticmethod
    def is_zero(a): return a == (0, 0)


# ----------------------------------------------------------------------------- curves (Jacobian)
class Curve:
    def __init__(self, F, b):
        self.F, self.b = F, b

    def inf(self):
        return None

    def dbl(self, p):
        if p is None:
            return None
        F = self.F
        X, Y, Z = p
        if F.is_zero(Y):
            return None
        XX = F.mul(X, X)
        YY = F.mul(Y, Y)
        S = F.mul(F.add(X, X), F.add(YY, YY))          # 4 X Y^2
        M = F.add(F.add(XX, XX), XX)                     # 3 X^2
        X3 = F.sub(F.mul(M, M), F.add(S, S))
        YYYY8 = F.mul(YY, YY)
        for _ in range(3):
            YYYY8 = F.add(YYYY8, YYYY8)
        Y3 = F.sub(F.mul(M, F.sub(S, X3)), YYYY8)
        Z3 = F.mul(F.add(Y, Y), Z)
        return (X3, Y3, Z3)

    def add(self, p, q):
        if p is None:
            return q
        if q is None:
            return p
        F = self.F
        X1, Y1, Z1 = p
        X2, Y2, Z2 = q
        Z1Z1, Z2Z2 = F.mul(Z1, Z1), F.mul(Z2, Z2)
        U1, U2 = F.mul(X1, Z2Z2), F.mul(X2, Z1Z1)
        S1 = F.mul(Y1, F.mul(Z2, Z2Z2))
        S2 = F.mul(Y2, F.mul(Z1, Z1Z1))
        if U1 == U2:
            return self.dbl(p) if S1 == S2 else None
        H = F.sub(U2, U1)
        rr = F.sub(S2, S1)
        HH = F.mul(H, H)
        HHH = F.mul(H, HH)
        V = F.mul(U1, HH)
        X3 = F.sub(F.sub(F.mul(rr, rr), HHH), F.add(V, V))
        Y3 = F.sub(F.mul(rr, F.sub(V, X3)), F.mul(S1, HHH))
        Z3 = F.mul(F.mul(Z1, Z2), H)
        return (X3, Y3, Z3)

    def from_aff(self, a):
        return None if a is None else (a[0], a[1], self.F.one)

    def to_aff(self, p):
        if p is None:
            return None
        F = self.F
        zi = F.inv(p[2])
        zi2 = F.mul(zi, zi)
        return (F.mul(p[0], zi2), F.mul(p[1], F.mul(zi2, zi)))

    def mul(self, p, k):
        k %= R
        acc = None
        for bit in bin(k)[2:] if k else "":
            acc = self.dbl(acc)
            if bit == "1":
                acc = self.add(acc, p)
        return acc

    def neg_aff(self, a):
        return None if a is None else (a[0], self.F.neg(a[1]))

    def on_curve(self, a):
        if a is None:
            return True
        F = self.F
        return F.mul(a[1], a[1]) == F.add(F.mul(F.mul(a[0], a[0]), a[0]), self.b)


E1 = Curve(Fq, 4)
E2 = Curve(Fq2, (4, 4))
G1 = (G1X, G1Y)
G2 = (G2X, G2Y)


def g1_mul_gen(k):
    return E1.to_aff(E1.mul(E1.from_aff(G1), k))


def g2_mul_gen(k):
    return E2.to_aff(E2.mul(E2.from_aff(G2), k))


# ----------------------------------------------------------------------------- encodings
def _be48(x):
    return x.to_bytes(48, "big")


def g1_uncompressed(a):
    if a is None:
        return bytes([0x40]) + bytes(95)
    return _be48(a[0]) + _be48(a[1])


def g2_uncompressed(a):
    if a is None:
        return bytes([0x40]) + bytes(191)
    return _be48(a[0][1]) + _be48(a[0][0]) + _be48(a[1][1]) + _be48(a[1][0])


def g1_from_uncompressed(b):
    if b[0] & 0x40:
        return None
    return (int.from_bytes(bytes([b[0] & 0x1F]) + b[1:48], "big"), int.from_bytes(b[48:96], "big"))


def g2_from_uncompressed(b):
    if b[0] & 0x40:
        return None
    x1 = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:96], "big")
    y1 = int.from_bytes(b[96:144], "big")
    y0 = int.from_bytes(b[144:192], "big")
    return ((x0, x1), (y0, y1))


def _largest(y):
    return y > (P - 1) // 2


def g1_compressed(a):
    if a is None:
        return bytes([0xC0]) + bytes(47)
    out = bytearray(_be48(a[0]))
    out[0] |= 0x80 | (0x20 if _largest(a[1]) else 0)
    return bytes(out)


def g2_compressed(a):
    if a is None:
        return bytes([0xC0]) + bytes(95)
    out = bytearray(_be48(a[0][1]) + _be48(a[0][0]))
    y0, y1 = a[1]
    largest = _largest(y1) if y1 != 0 else _largest(y0)
    out[0] |= 0x80 | (0x20 if largest else 0)
    return bytes(out)


def fr_le(x):
    return (x % R).to_bytes(32, "little")


# ----------------------------------------------------------------------------- evaluation domain
GENERATOR = 7
ROOT_OF_UNITY = pow(GENERATOR, (R - 1) >> 32, R)


def omega(log_n):
    return pow(ROOT_OF_UNITY, 1 << (32 - log_n), R)


def dft(a, w):
    """Iterative radix-2 Cooley-Tukey (decimation in frequency, Gentleman-Sande) then bit reversal."""
    n = len(a)
    a = list(a)
    m = n
    while m > 1:
        half = m // 2
        wm = pow(w, n // m, R)
        for k in range(0, n, m):
            t = 1
            for j in range(half):
                u, v = a[k + j], a[k + j + half]
                a[k + j] = (u + v) % R
                a[k + j + half] = ((u - v) * t) % R
                t = (t * wm) % R
        m = half
    bits = n.bit_length() - 1
    out = [0] * n
    for i in range(n):
        out[int(format(i, "0%db" % bits)[::-1], 2) if bits else 0] = a[i]
    return out


def domain(a, log_n, kind):
    n = 1 << log_n
    w = omega(log_n)
    if kind == 0:
        return dft(a, w)
    if kind == 1:
        ninv = pow(n, R - 2, R)
        return [(x * ninv) % R for x in dft(a, pow(w, R - 2, R))]
    if kind == 2:
        return dft([(x * pow(GENERATOR, i, R)) % R for i, x in enumerate(a)], w)
    if kind == 3:
        ninv = pow(n, R - 2, R)
        gi = pow(GENERATOR, R - 2, R)
        return [(x * ninv * pow(gi, i, R)) % R for i, x in enumerate(dft(a, pow(w, R - 2, R)))]
    raise ValueError(kind)


# ----------------------------------------------------------------------------- multiexp (naive)
def msm(curve, bases, scalars):
    acc = None
    for b, k in zip(bases, scalars):
        acc = curve.add(acc, curve.mul(curve.from_aff(b), k))
    return curve.to_aff(acc)


# ----------------------------------------------------------------------------- Groth16 (bellman)
class Circuit:
    """rows: list of (A, B, C), each a list of (var, coeff).  Vars 0..n_in-1 inputs (0 = ONE)."""

    def __init__(self, n_in, n_aux, rows):
        self.n_in, self.n_aux, self.rows = n_in, n_aux, rows

    def satisfied(self, z):
        ev = lambda lc: sum(c * z[v] for v, c in lc) % R
        return all(ev(a) * ev(b) % R == ev(c) for a, b, c in self.rows)


def keygen(circ, toxic):
    tau, alpha, beta, gamma, delta = toxic
    n = len(circ.rows)
    rows_total = n + circ.n_in
    log_d = max(0, (rows_total - 1).bit_length())
    d = 1 << log_d
    powers = [pow(tau, i, R) for i in range(d)]
    lag = domain(powers, log_d, 1)
    t_tau = (pow(tau, d, R) - 1) % R
    dinv, ginv = pow(delta, R - 2, R), pow(gamma, R - 2, R)
    nv = circ.n_in + circ.n_aux
    at, bt, ct = [0] * nv, [0] * nv, [0] * nv
    a_aux_den, b_in_den, b_aux_den = [0] * circ.n_aux, [0] * circ.n_in, [0] * circ.n_aux
    for j, (A, B, C) in enumerate(circ.rows):
        for v, c in A:
            at[v] = (at[v] + c * lag[j]) % R
            if v >= circ.n_in:
                a_aux_den[v - circ.n_in] = 1
        for v, c in B:
            bt[v] = (bt[v] + c * lag[j]) % R
            if v < circ.n_in:
                b_in_den[v] = 1
            else:
                b_aux_den[v - circ.n_in] = 1
        for v, c in C:
            ct[v] = (ct[v] + c * lag[j]) % R
    for i in range(circ.n_in):
        at[i] = (at[i] + lag[n + i]) % R
    pk = dict(d=d, log_d=log_d, at=at, bt=bt, ct=ct, a_aux_den=a_aux_den, b_in_den=b_in_den,
              b_aux_den=b_aux_den, toxic=toxic)
    pk["h"] = [g1_mul_gen(powers[i] * t_tau * dinv) for i in range(d - 1)]
    ext = [(beta * at[v] + alpha * bt[v] + ct[v]) % R for v in range(nv)]
    pk["ic"] = [g1_mul_gen(ext[v] * ginv) for v in range(circ.n_in)]
    pk["l"] = [g1_mul_gen(ext[v] * dinv) for v in range(circ.n_in, nv)]
    pk["a"] = [g1_mul_gen(at[v]) for v in range(nv) if at[v]]
    pk["b_g1"] = [g1_mul_gen(bt[v]) for v in range(nv) if bt[v]]
    pk["b_g2"] = [g2_mul_gen(bt[v]) for v in range(nv) if bt[v]]
    pk["alpha_g1"], pk["beta_g1"], pk["delta_g1"] = g1_mul_gen(alpha), g1_mul_gen(beta), g1_mul_gen(delta)
    pk["beta_g2"], pk["gamma_g2"], pk["delta_g2"] = g2_mul_gen(beta), g2_mul_gen(gamma), g2_mul_gen(delta)
    return pk


def prove(pk, circ, z, r, s):
    d, log_d, n = pk["d"], pk["log_d"], len(circ.rows)
    ev = lambda lc: sum(c * z[v] for v, c in lc) % R
    a = [ev(A) for A, _, _ in circ.rows] + [z[i] for i in range(circ.n_in)]
    b = [ev(B) for _, B, _ in circ.rows] + [0] * circ.n_in
    c = [ev(C) for _, _, C in circ.rows] + [0] * circ.n_in
    pad = d - len(a)
    a, b, c = a + [0] * pad, b + [0] * pad, c + [0] * pad
    a = domain(domain(a, log_d, 1), log_d, 2)
    b = domain(domain(b, log_d, 1), log_d, 2)
    c = domain(domain(c, log_d, 1), log_d, 2)
    zinv = pow((pow(GENERATOR, d, R) - 1) % R, R - 2, R)
    hev = [((x * y - w) * zinv) % R for x, y, w in zip(a, b, c)]
    h = domain(hev, log_d, 3)[: d - 1]
    n_in = circ.n_in
    inputs, aux = z[:n_in], z[n_in:]
    H = msm(E1, pk["h"], h)
    L = msm(E1, pk["l"], aux)
    ka = inputs + [aux[i] for i in range(circ.n_aux) if pk["a_aux_den"][i]]
    kb = [inputs[i] for i in range(n_in) if pk["b_in_den"][i]] + \
         [aux[i] for i in range(circ.n_aux) if pk["b_aux_den"][i]]
    assert len(ka) == len(pk["a"]) and len(kb) == len(pk["b_g1"])
    As = E1.from_aff(msm(E1, pk["a"], ka))
    B1 = E1.from_aff(msm(E1, pk["b_g1"], kb))
    B2 = E2.from_aff(msm(E2, pk["b_g2"], kb))
    J1 = E1.from_aff
    A = E1.add(E1.add(J1(pk["alpha_g1"]), As), E1.mul(J1(pk["delta_g1"]), r))
    B = E2.add(E2.add(E2.from_aff(pk["beta_g2"]), B2), E2.mul(E2.from_aff(pk["delta_g2"]), s))
    C = E1.mul(J1(pk["delta_g1"]), r * s)
    for t in (E1.mul(J1(pk["alpha_g1"]), s), E1.mul(J1(pk["beta_g1"]), r), E1.mul(As, s), E1.mul(B1, r),
              E1.from_aff(H), E1.from_aff(L)):
        C = E1.add(C, t)
    Aa, Ba, Ca = E1.to_aff(A), E2.to_aff(B), E1.to_aff(C)
    proof = g1_compressed(Aa) + g2_compressed(Ba) + g1_compressed(Ca)
    raw = g1_uncompressed(Aa) + g2_uncompressed(Ba) + g1_uncompressed(Ca)
    return proof, raw, h


# ----------------------------------------------------------------------------- pairing (py_ecc style)
# Fq12 = Fq[w] / (w^12 - 2 w^6 + 2); Fq2 -> Fq12 via u -> w^6 - 1; twist (x, y) -> (x/w^2, y/w^3)
def f12_mul(a, b):
    t = [0] * 23
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                t[i + j] += x * y
    for k in range(22, 11, -1):
        t[k - 6] += 2 * t[k]
        t[k - 12] -= 2 * t[k]
    return [x % P for x in t[:12]]


def f12_pow(a, e):
    r = [1] + [0] * 11
    for bit in bin(e)[2:]:
        r = f12_mul(r, r)
        if bit == "1":
            r = f12_mul(r, a)
    return r


def f12_inv_w():
    m2inv = pow(P - 2, P - 2, P)
    r = [0] * 12
    r[11] = m2inv
    r[5] = (-2 * m2inv) % P
    return r


def _emb(x):
    r = [0] * 12
    r[0] = (x[0] - x[1]) % P
    r[6] = x[1]
    return r


def miller_loop(Q, Pp):
    if Q is None or Pp is None:
        return [1] + [0] * 11
    wi = f12_inv_w()
    wi2 = f12_mul(wi, wi)
    wi3 = f12_mul(wi2, wi)
    xP = [Pp[0]] + [0] * 11
    yP = [Pp[1]] + [0] * 11

    def line(Rp, slope):
        m12 = f12_mul(_emb(slope), wi)
        xr = f12_mul(_emb(Rp[0]), wi2)
        yr = f12_mul(_emb(Rp[1]), wi3)
        a = f12_mul(m12, [(u - v) % P for u, v in zip(xP, xr)])
        return [(u - (v - w)) % P for u, v, w in zip(a, yP, yr)]

    ate = 0xD201000000010000
    Rp = Q
    f = [1] + [0] * 11
    for i in range(62, -1, -1):
        x, y = Rp
        slope = Fq2.mul(Fq2.mul((3, 0), Fq2.mul(x, x)), Fq2.inv(Fq2.add(y, y)))
        f = f12_mul(f12_mul(f, f), line(Rp, slope))
        nx = Fq2.sub(Fq2.mul(slope, slope), Fq2.add(x, x))
        Rp = (nx, Fq2.sub(Fq2.mul(slope, Fq2.sub(x, nx)), y))
        if (ate >> i) & 1:
            x, y = Rp
            s2 = Fq2.mul(Fq2.sub(Q[1], y), Fq2.inv(Fq2.sub(Q[0], x)))
            f = f12_mul(f, line(Rp, s2))
            ax = Fq2.sub(Fq2.sub(Fq2.mul(s2, s2), x), Q[0])
            Rp = (ax, Fq2.sub(Fq2.mul(s2, Fq2.sub(x, ax)), y))
    return f


def verify(pk, inputs, raw):
    A = g1_from_uncompressed(raw[:96])
    B = g2_from_uncompressed(raw[96:288])
    C = g1_from_uncompressed(raw[288:384])
    IC = msm(E1, pk["ic"], inputs)
    f = miller_loop(B, A)
    f = f12_mul(f, miller_loop(pk["beta_g2"], E1.neg_aff(pk["alpha_g1"])))
    f = f12_mul(f, miller_loop(pk["gamma_g2"], E1.neg_aff(IC)))
    f = f12_mul(f, miller_loop(pk["delta_g2"], E1.neg_aff(C)))
    return f12_pow(f, (P ** 12 - 1) // R) == [1] + [0] * 11


# ----------------------------------------------------------------------------- deterministic inputs
class SplitMix64:
    def __init__(self, seed):
        self.s = seed & 0xFFFFFFFFFFFFFFFF

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        return z ^ (z >> 31)

    def fr(self):
        v = 0
        for i in range(4):
            v |= self.next() << (64 * i)
        return v % R
