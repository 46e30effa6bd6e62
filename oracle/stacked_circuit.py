"""stacked_circuit.py -- TEST INFRASTRUCTURE ONLY (the checker of SURVEY.md §8(f)#3, never the product).

A CPU restatement, with witness values, of the constraint system the reference synthesises for the stacked
PoRep circuit (libs/storage/include/nil/filecoin/storage/proofs/porep/stacked/circuit/proof.hpp:98-165
StackedCircuit::synthesize, params.hpp:93-238 Proof::synthesize) and of the gadgets it calls.  The gadget
code lives in third-party crates the reference names but does not vendor (bellman / bellperson: boolean,
uint32, multieq, sha256, num, multipack; rust-fil-proofs storage-proofs-core: insertion, por, encode,
create_label; neptune: the Poseidon circuit); pinned version: none (the crypto3 zk submodule is empty).
This file restates their published algorithms.

What pins the layout.  The reference's own tests assert constraint counts (no witness vectors exist):
  * libs/storage/test/porep/stacked/circuit/hash.cpp:77      hash_single_column (Poseidon, 11 inputs): 598
  * libs/storage/test/core/components/por.cpp:89-172         PoR circuits: SHA-256 base 2/4/8 = 272,295 /
    216,258 / 250,987; Poseidon base 2/4/8 = 1,887 / 1,164 / 1,063; 8-2 = 1,377; 8-4-2 = 1,764; 8-8 = 1,593;
    8-8-2 = 1,907 (and the private variants, one fewer)
  * libs/storage/test/porep/stacked/circuit/proof.cpp:137-155  the stacked circuit, 2 layers, 1 challenge,
    8 x base-tree-count nodes: 22 inputs; Poseidon base 2 / base 8 / 8-4 / 8-4-2 = 1,206,212 / 1,199,620 /
    1,296,576 / 1,346,982 constraints
tests/test_cpu_stacked_circuit.py asserts every one of those numbers against this restatement.  The SHA-256
gadget is also pinned by bellman's own published count (25,840 per compression of 512 variable bits).
Variable ORDER and the exact linear combinations beyond those counts are parity-unpinned: where a gadget's
internals are not fixed by a count (the Poseidon circuit's round layout, the order of insert_8's picks) the
choice below is stated.

Representation: LC = list of (var, coeff); var >= 0 is aux index, var < 0 is input ~var (input 0 = ONE).
Every LC is canonicalised (merged, sorted, zeros dropped) when the constraint is recorded.
"""
from poseidon_ref import R, Poseidon, ROUNDS

ONE = ~0  # input 0
CAPACITY = 254  # Fr::CAPACITY for BLS12-381


# ------------------------------------------------------------------------------------------ constraint system
class CS:
    """bellman TestConstraintSystem: alloc / alloc_input / enforce, with values."""

    def __init__(self, with_constraints=True):
        self.inputs = [1]
        self.aux = []
        self.rows = []  # (A, B, C) canonical LCs
        self.n_constraints = 0
        self.keep = with_constraints

    def alloc(self, value):
        self.aux.append(value % R)
        return len(self.aux) - 1

    def alloc_input(self, value):
        self.inputs.append(value % R)
        return ~(len(self.inputs) - 1)

    def enforce(self, a, b, c):
        self.n_constraints += 1
        if self.keep:
            self.rows.append((canon(a), canon(b), canon(c)))

    def value(self, var):
        return self.inputs[~var] if var < 0 else self.aux[var]

    def lc_value(self, lc):
        return sum(self.value(v) * k for v, k in lc) % R

    def is_satisfied(self):
        for i, (a, b, c) in enumerate(self.rows):
            if self.lc_value(a) * self.lc_value(b) % R != self.lc_value(c):
                return i
        return None

    # z = ONE ++ inputs ++ aux (the boundary's variable order)
    def z_index(self, var):
        return ~var if var < 0 else len(self.inputs) + var

    def to_csr(self):
        """3 x (row_ptr, cols, coeffs) over z = inputs ++ aux, the rows in synthesis order."""
        out = []
        for m in range(3):
            rp, cols, cos = [0], [], []
            for row in self.rows:
                for v, k in row[m]:
                    cols.append(self.z_index(v))
                    cos.append(k)
                rp.append(len(cols))
            out.append((rp, cols, cos))
        return out

    def z(self):
        return self.inputs + self.aux


def canon(lc):
    d = {}
    for v, k in lc:
        d[v] = (d.get(v, 0) + k) % R
    # inputs (negative vars) first in input order, then aux: the z order
    return sorted(((v, k) for v, k in d.items() if k), key=lambda vk: (vk[0] >= 0, ~vk[0] if vk[0] < 0 else vk[0]))


def lc_scale(lc, k):
    return [(v, c * k % R) for v, c in lc]


# ------------------------------------------------------------------------------------------ Boolean (bellman)
# (kind, var, val): kind 0 = Constant(val), 1 = Is(var), 2 = Not(var); val = the Boolean's logical value
def const(b):
    return (0, None, b & 1)


FALSE, TRUE = const(0), const(1)


def is_const(b):
    return b[0] == 0


def bnot(b):
    if b[0] == 0:
        return (0, None, 1 - b[2])
    return (3 - b[0], b[1], 1 - b[2])


def blc(b, coeff=1):
    """Boolean::lc(one, coeff)"""
    if b[0] == 0:
        return [(ONE, coeff)] if b[2] else []
    if b[0] == 1:
        return [(b[1], coeff)]
    return [(ONE, coeff), (b[1], (R - coeff) % R)]


def bvarval(b):
    """value of the underlying variable of an Is / Not Boolean"""
    return b[2] if b[0] == 1 else 1 - b[2]


def alloc_bit(cs, value):
    """AllocatedBit::alloc: boolean constraint (1 - a) * a = 0"""
    v = cs.alloc(value)
    cs.enforce([(ONE, 1), (v, R - 1)], [(v, 1)], [])
    return (1, v, value & 1)


def abit_xor(cs, a, b):
    """AllocatedBit::xor over the variables of Is(a), Is(b): (a + a) * b = a + b - c"""
    av, bv = bvarval(a), bvarval(b)
    c = cs.alloc(av ^ bv)
    cs.enforce([(a[1], 2)], [(b[1], 1)], [(a[1], 1), (b[1], 1), (c, R - 1)])
    return c, av ^ bv


def abit_and(cs, a, b):
    av, bv = bvarval(a), bvarval(b)
    c = cs.alloc(av & bv)
    cs.enforce([(a[1], 1)], [(b[1], 1)], [(c, 1)])
    return (1, c, av & bv)


def abit_and_not(cs, a, b):
    """a AND NOT b over variables: a * (1 - b) = c"""
    av, bv = bvarval(a), bvarval(b)
    c = cs.alloc(av & (1 - bv))
    cs.enforce([(a[1], 1)], [(ONE, 1), (b[1], R - 1)], [(c, 1)])
    return (1, c, av & (1 - bv))


def abit_nor(cs, a, b):
    """NOT a AND NOT b over variables: (1 - a) * (1 - b) = c"""
    av, bv = bvarval(a), bvarval(b)
    c = cs.alloc((1 - av) & (1 - bv))
    cs.enforce([(ONE, 1), (a[1], R - 1)], [(ONE, 1), (b[1], R - 1)], [(c, 1)])
    return (1, c, (1 - av) & (1 - bv))


def bxor(cs, a, b):
    """Boolean::xor"""
    if a == FALSE:
        return b
    if b == FALSE:
        return a
    if a == TRUE:
        return bnot(b)
    if b == TRUE:
        return bnot(a)
    if a[0] != b[0]:  # Is with Not: NOT(is XOR not's variable), the Is operand first
        c, cv = abit_xor(cs, a, b) if a[0] == 1 else abit_xor(cs, b, a)
        return (2, c, 1 - cv)
    c, cv = abit_xor(cs, a, b)  # Is/Is or Not/Not: the variables' xor is the logical xor
    return (1, c, cv)


def band(cs, a, b):
    """Boolean::and"""
    if a == FALSE or b == FALSE:
        return FALSE
    if a == TRUE:
        return b
    if b == TRUE:
        return a
    if a[0] == 1 and b[0] == 2:
        return abit_and_not(cs, a, b)
    if a[0] == 2 and b[0] == 1:
        return abit_and_not(cs, b, a)
    if a[0] == 2 and b[0] == 2:
        return abit_nor(cs, a, b)
    return abit_and(cs, a, b)


def sha256_ch(cs, a, b, c):
    """Boolean::sha256_ch: (a and b) xor ((not a) and c)"""
    val = (a[2] & b[2]) ^ ((1 - a[2]) & c[2])
    if is_const(a) and is_const(b) and is_const(c):
        return const(val)
    if a == FALSE:
        return c
    if b == FALSE:
        return band(cs, bnot(a), c)
    if c == FALSE:
        return band(cs, a, b)
    if c == TRUE:
        return bnot(band(cs, a, bnot(b)))
    if b == TRUE:
        return bnot(band(cs, bnot(a), bnot(c)))
    ch = cs.alloc(val)
    # a (b - c) = ch - c
    cs.enforce(blc(b) + lc_scale(blc(c), R - 1), blc(a), [(ch, 1)] + lc_scale(blc(c), R - 1))
    return (1, ch, val)


def sha256_maj(cs, a, b, c):
    """Boolean::sha256_maj: (a and b) xor (a and c) xor (b and c)"""
    val = (a[2] & b[2]) ^ (a[2] & c[2]) ^ (b[2] & c[2])
    if is_const(a) and is_const(b) and is_const(c):
        return const(val)
    if a == FALSE:
        return band(cs, b, c)
    if b == FALSE:
        return band(cs, a, c)
    if c == FALSE:
        return band(cs, a, b)
    if c == TRUE:
        return bnot(band(cs, bnot(a), bnot(b)))
    if b == TRUE:
        return bnot(band(cs, bnot(a), bnot(c)))
    if a == TRUE:
        return bnot(band(cs, bnot(b), bnot(c)))
    maj = cs.alloc(val)
    bc = band(cs, b, c)
    # (2bc - b - c) * a = bc - maj
    cs.enforce(blc(bc, 2) + lc_scale(blc(b), R - 1) + lc_scale(blc(c), R - 1), blc(a), blc(bc) + [(maj, R - 1)])
    return (1, maj, val)


# ------------------------------------------------------------------------------------------ UInt32 (bellman)
# a UInt32 is a list of 32 Booleans, bits[0] = least significant
def u32_const(x):
    return [const((x >> i) & 1) for i in range(32)]


def u32_from_bits_be(bits):
    return list(reversed(bits))


def u32_into_bits_be(u):
    return list(reversed(u))


def u32_value(u):
    return sum(b[2] << i for i, b in enumerate(u))


def rotr(u, k):
    return [u[(i + k) % 32] for i in range(32)]


def shr(u, k):
    return [u[i + k] if i + k < 32 else FALSE for i in range(32)]


def u32_xor(cs, a, b):
    return [bxor(cs, x, y) for x, y in zip(a, b)]


class MultiEq:
    """bellman MultiEq: equalities of <= CAPACITY - 1 packed bits share one constraint"""

    def __init__(self, cs):
        self.cs, self.bits, self.lhs, self.rhs = cs, 0, [], []

    def accumulate(self):
        self.cs.enforce(self.lhs, [(ONE, 1)], self.rhs)
        self.lhs, self.rhs, self.bits = [], [], 0

    def enforce_equal(self, nbits, lhs, rhs):
        if CAPACITY <= self.bits + nbits:
            self.accumulate()
        k = 1 << self.bits
        self.lhs += lc_scale(lhs, k)
        self.rhs += lc_scale(rhs, k)
        self.bits += nbits

    def close(self):
        if self.bits > 0:
            self.accumulate()


def addmany(cs, me, ops):
    """UInt32::addmany"""
    assert 2 <= len(ops) <= 10
    total = sum(u32_value(o) for o in ops)
    if all(is_const(b) for o in ops for b in o):
        return u32_const(total & 0xFFFFFFFF)
    lc = []
    for o in ops:
        for i, b in enumerate(o):
            lc += blc(b, 1 << i)
    nb = (len(ops) * 0xFFFFFFFF).bit_length()
    res, rlc = [], []
    for i in range(nb):
        b = alloc_bit(cs, (total >> i) & 1)
        res.append(b)
        rlc.append((b[1], 1 << i))
    me.enforce_equal(nb, lc, rlc)
    return res[:32]


IV = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]
K = [0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
     0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
     0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
     0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
     0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
     0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
     0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
     0xc67178f2]


def sha256_compression(cs, bits, H):
    """bellman sha256_compression_function (one MultiEq per compression, deferred a / e additions)"""
    assert len(bits) == 512 and len(H) == 8
    w = [u32_from_bits_be(bits[32 * i:32 * i + 32]) for i in range(16)]
    me = MultiEq(cs)
    for i in range(16, 64):
        s0 = u32_xor(cs, rotr(w[i - 15], 7), rotr(w[i - 15], 18))
        s0 = u32_xor(cs, s0, shr(w[i - 15], 3))
        s1 = u32_xor(cs, rotr(w[i - 2], 17), rotr(w[i - 2], 19))
        s1 = u32_xor(cs, s1, shr(w[i - 2], 10))
        w.append(addmany(cs, me, [w[i - 16], s0, w[i - 7], s1]))

    def compute(m, others):
        return m[1] if m[0] == "c" else addmany(cs, me, m[1] + others)

    a, b, c, d = ("c", H[0]), H[1], H[2], H[3]
    e, f, g, h = ("c", H[4]), H[5], H[6], H[7]
    for i in range(64):
        ne = compute(e, [])
        s1 = u32_xor(cs, rotr(ne, 6), rotr(ne, 11))
        s1 = u32_xor(cs, s1, rotr(ne, 25))
        ch = [sha256_ch(cs, x, y, z) for x, y, z in zip(ne, f, g)]
        t1 = [h, s1, ch, u32_const(K[i]), w[i]]
        na = compute(a, [])
        s0 = u32_xor(cs, rotr(na, 2), rotr(na, 13))
        s0 = u32_xor(cs, s0, rotr(na, 22))
        mj = [sha256_maj(cs, x, y, z) for x, y, z in zip(na, b, c)]
        h, g, f = g, f, ne
        e = ("d", t1 + [d])
        d, c, b = c, b, na
        a = ("d", t1 + [s0, mj])
    h0 = compute(a, [H[0]])
    h1 = addmany(cs, me, [H[1], b])
    h2 = addmany(cs, me, [H[2], c])
    h3 = addmany(cs, me, [H[3], d])
    h4 = compute(e, [H[4]])
    h5 = addmany(cs, me, [H[5], f])
    h6 = addmany(cs, me, [H[6], g])
    h7 = addmany(cs, me, [H[7], h])
    me.close()
    return [h0, h1, h2, h3, h4, h5, h6, h7]


def sha256(cs, bits):
    """bellman sha256: padding with constant bits, then one compression per block; big-endian output bits"""
    assert len(bits) % 8 == 0
    n = len(bits)
    p = list(bits) + [TRUE]
    while (len(p) + 64) % 512:
        p.append(FALSE)
    p += [const((n >> i) & 1) for i in range(63, -1, -1)]
    cur = [u32_const(x) for x in IV]
    for k in range(0, len(p), 512):
        cur = sha256_compression(cs, p[k:k + 512], cur)
    return [b for u in cur for b in u32_into_bits_be(u)]


# ------------------------------------------------------------------------------------------ num / multipack
def alloc_num(cs, value):
    return cs.alloc(value)


def inputize(cs, var):
    """AllocatedNum::inputize: input * 1 = var"""
    inp = cs.alloc_input(cs.value(var))
    cs.enforce([(inp, 1)], [(ONE, 1)], [(var, 1)])
    return inp


def to_bits_le(cs, var):
    """AllocatedNum::to_bits_le (non-strict): 255 AllocatedBits LSB first, then 0 * 0 = sum 2^i b_i - x"""
    x = cs.value(var)
    bits = [alloc_bit(cs, (x >> i) & 1) for i in range(255)]
    lc = [(b[1], 1 << i) for i, b in enumerate(bits)] + [(var, R - 1)]
    cs.enforce([], [], lc)
    return bits


def reverse_bit_numbering(bits):
    """storage-proofs-core util::reverse_bit_numbering: pad to whole bytes, reverse each byte's bits"""
    b = list(bits)
    while len(b) % 8:
        b.append(FALSE)
    out = []
    for k in range(0, len(b), 8):
        out += list(reversed(b[k:k + 8]))
    return out


def pack_bits(cs, bits):
    """storage-proofs-core multipack::pack_bits: the first CAPACITY bits -> one AllocatedNum"""
    lc, val = [], 0
    for i, b in enumerate(bits[:CAPACITY]):
        lc += blc(b, 1 << i)
        val |= b[2] << i
    v = cs.alloc(val)
    cs.enforce(lc, [(ONE, 1)], [(v, 1)])
    return v


def pack_into_inputs(cs, bits):
    """bellman multipack::pack_into_inputs: chunks of CAPACITY bits -> inputs"""
    out = []
    for k in range(0, len(bits), CAPACITY):
        lc, val = [], 0
        for i, b in enumerate(bits[k:k + CAPACITY]):
            lc += blc(b, 1 << i)
            val |= b[2] << i
        inp = cs.alloc_input(val)
        cs.enforce(lc, [(ONE, 1)], [(inp, 1)])
        out.append(inp)
    return out


def uint64_alloc(cs, value):
    """bellman UInt64::alloc: 64 AllocatedBits, LSB first"""
    return [alloc_bit(cs, (value >> i) & 1) for i in range(64)]


def equal(cs, a, b):
    """storage-proofs-core constraint::equal: a * 1 = b"""
    cs.enforce([(a, 1)], [(ONE, 1)], [(b, 1)])


def add(cs, a, b):
    """constraint::add (encode): (a + b) * 1 = sum"""
    s = cs.alloc(cs.value(a) + cs.value(b))
    cs.enforce([(a, 1), (b, 1)], [(ONE, 1)], [(s, 1)])
    return s


# ------------------------------------------------------------------------------------------ insertion (fil-proofs)
def pick(cs, cond, a, b):
    """(b - a) * cond = b - c: c = cond ? a : b"""
    c = cs.alloc(cs.value(a) if cond[2] else cs.value(b))
    cs.enforce([(b, 1), (a, R - 1)], blc(cond), [(b, 1), (c, R - 1)])
    return c


def insert(cs, element, bits, elements):
    size = len(elements) + 1
    assert 1 << len(bits) == size
    if size == 2:
        return [pick(cs, bits[0], elements[0], element), pick(cs, bits[0], element, elements[0])]
    if size == 4:
        b0, b1 = bits
        a, b, c, d = element, *elements
        p0_x0 = pick(cs, b0, b, a)
        p0 = pick(cs, b1, b, p0_x0)
        p1_x0 = pick(cs, b0, a, b)
        p1 = pick(cs, b1, c, p1_x0)
        p2_x1 = pick(cs, b0, d, a)
        p2 = pick(cs, b1, p2_x1, c)
        p3_x1 = pick(cs, b0, a, d)
        p3 = pick(cs, b1, p3_x1, d)
        return [p0, p1, p2, p3]
    if size == 8:
        b0, b1, b2 = bits
        a, b, c, d, e, f, g, h = element, *elements
        nor01 = abit_nor(cs, b0, b1)
        and01 = abit_and(cs, b0, b1)
        p0_xx0 = pick(cs, nor01, a, b)
        p0 = pick(cs, b2, b, p0_xx0)
        p1_x00 = pick(cs, b0, a, b)
        p1_xx0 = pick(cs, b1, c, p1_x00)
        p1 = pick(cs, b2, c, p1_xx0)
        p2_x10 = pick(cs, b0, d, a)
        p2_xx0 = pick(cs, b1, p2_x10, c)
        p2 = pick(cs, b2, d, p2_xx0)
        p3_xx0 = pick(cs, and01, a, d)
        p3 = pick(cs, b2, e, p3_xx0)
        p4_xx1 = pick(cs, nor01, a, f)
        p4 = pick(cs, b2, p4_xx1, e)
        p5_x01 = pick(cs, b0, a, f)
        p5_xx1 = pick(cs, b1, g, p5_x01)
        p5 = pick(cs, b2, p5_xx1, f)
        p6_x11 = pick(cs, b0, h, a)
        p6_xx1 = pick(cs, b1, p6_x11, g)
        p6 = pick(cs, b2, p6_xx1, g)
        p7_xx1 = pick(cs, and01, a, h)
        p7 = pick(cs, b2, p7_xx1, h)
        return [p0, p1, p2, p3, p4, p5, p6, p7]
    raise ValueError("insert: arity must be 2, 4 or 8")


# ------------------------------------------------------------------------------------------ Poseidon circuit
_POSEIDON = {}


def poseidon_params(arity):
    if arity not in _POSEIDON:
        _POSEIDON[arity] = Poseidon(arity)
    return _POSEIDON[arity]


def poseidon_constraints(arity):
    """the count this layout produces: 3 per S-box of the first round (the constant domain-tag S-box is free),
    4 per later S-box (the input linear combination is allocated, then squared, squared, multiplied), 1 for
    the allocated digest"""
    t = arity + 1
    r_f, r_p = ROUNDS[arity]
    return 3 * (t - 1) + 4 * ((r_f - 1) * t + r_p) + 1


def poseidon_hash_circuit(cs, inputs, arity):
    """neptune poseidon_hash circuit as the counts above pin it (598 for arity 11: hash.cpp:77; arity 2 / 4 /
    8 from the PoR counts).  Round layout (parity-unpinned beyond the count): the literal permutation of
    poseidon_ref (ARK, S-box, state' = state * M); state elements are linear combinations; every S-box
    after the first round first allocates its input LC."""
    P = poseidon_params(arity)
    t = P.t
    assert len(inputs) == arity
    st = [([], P.tag)] + [([(x, 1)], cs.value(x)) for x in inputs]  # (lc without ONE term, value incl. const)
    cst = [P.tag] + [0] * arity  # constant part of each element's LC
    k = 0
    half = P.r_f // 2
    for rnd in range(P.r_f + P.r_p):
        for i in range(t):
            cst[i] = (cst[i] + P.rc[k + i]) % R
            st[i] = (st[i][0], (st[i][1] + P.rc[k + i]) % R)
        k += t
        full = rnd < half or rnd >= half + P.r_p
        for i in (range(t) if full else [0]):
            lc, val = st[i]
            if not lc:  # constant (the domain tag in the first round)
                st[i] = ([], pow(val, 5, R))
                cst[i] = st[i][1]
                continue
            xlc = lc + ([(ONE, cst[i])] if cst[i] else [])
            if rnd == 0:
                v_lc = xlc
            else:
                v = cs.alloc(val)
                cs.enforce(xlc, [(ONE, 1)], [(v, 1)])
                v_lc = [(v, 1)]
            l2 = cs.alloc(val * val)
            cs.enforce(v_lc, v_lc, [(l2, 1)])
            l4 = cs.alloc(pow(val, 4, R))
            cs.enforce([(l2, 1)], [(l2, 1)], [(l4, 1)])
            l5 = cs.alloc(pow(val, 5, R))
            cs.enforce([(l4, 1)], v_lc, [(l5, 1)])
            st[i] = ([(l5, 1)], pow(val, 5, R))
            cst[i] = 0
        new, ncst = [], []
        for j in range(t):
            lc, val, c = {}, 0, 0
            for i in range(t):
                m = P.m[i][j]
                for v, q in st[i][0]:
                    lc[v] = (lc.get(v, 0) + q * m) % R
                val += st[i][1] * m
                c += cst[i] * m
            new.append(([(v, q) for v, q in lc.items() if q], val % R))
            ncst.append(c % R)
        st, cst = new, ncst
    lc, val = st[1]
    out = cs.alloc(val)
    cs.enforce(lc + ([(ONE, cst[1])] if cst[1] else []), [(ONE, 1)], [(out, 1)])
    return out


# ------------------------------------------------------------------------------------------ hashers
def sha256_hash_leaves(cs, leaves):
    """storage-proofs-core Sha256Function::hash_multi_leaf_circuit / hash2_circuit: each leaf's 255-bit LE
    decomposition padded to whole bytes and bit-reversed per byte, concatenated, SHA-256, the first 254 output
    bits (LSB first per byte) packed"""
    pre = []
    for x in leaves:
        pre += reverse_bit_numbering(to_bits_le(cs, x))
    out = sha256(cs, pre)
    le = []
    for k in range(0, 256, 8):
        le += list(reversed(out[k:k + 8]))
    return pack_bits(cs, le)


def hash_multi_leaf(cs, hasher, arity, leaves):
    if hasher == "sha256":
        return sha256_hash_leaves(cs, leaves)
    return poseidon_hash_circuit(cs, leaves, arity)


# ------------------------------------------------------------------------------------------ PoR (fil-proofs)
def tree_levels(leaves, shape):
    """per-level arities of a (base, sub, top) tree over `leaves` leaves (rust-fil-proofs base tree count =
    sub * top trees of leaves / (sub * top) leaves)"""
    base, sub, top = shape
    per_base = leaves // ((sub or 1) * (top or 1))
    levels = []
    n = per_base
    while n > 1:
        levels.append(base)
        n //= base
    if sub:
        levels.append(sub)
    if top:
        levels.append(top)
    return levels


def por_synthesize(cs, leaf, index, siblings, root, levels, hasher, private=True):
    """PoRCircuit::synthesize (core/components/por.hpp): per level the index bits (AllocatedBit), the
    sibling allocations, insert, hash; then the path bits packed into one public input, and computed root ==
    root.  siblings[level] = the arity - 1 sibling values in position order."""
    cur = leaf
    path_bits = []
    shift = 0
    for lvl, arity in enumerate(levels):
        nb = arity.bit_length() - 1
        pos = (index >> shift) & (arity - 1)
        bits = [alloc_bit(cs, (pos >> i) & 1) for i in range(nb)]
        path_bits += bits
        nums = [cs.alloc(v) for v in siblings[lvl]]
        cur = hash_multi_leaf(cs, hasher, arity, insert(cs, cur, bits, nums))
        shift += nb
    pack_into_inputs(cs, path_bits)
    equal(cs, cur, root)
    if not private:
        inputize(cs, root)
    return cur


# ------------------------------------------------------------------------------------------ create_label
def create_label_circuit(cs, replica_id_bits, parents, layer, node_bits):
    """rust-fil-proofs stacked/circuit/create_label.rs: replica_id (256 bits) | layer u32 BE | node u64 BE |
    zeros to 64 bytes | 37 parents x 256 bits -> SHA-256 -> 254 bits packed"""
    assert len(parents) == 37
    m = list(replica_id_bits)
    while len(m) < 256:
        m.append(FALSE)
    m += u32_into_bits_be(u32_const(layer))
    m += list(reversed(node_bits))  # UInt64::to_bits_be
    while len(m) < 512:
        m.append(FALSE)
    for p in parents:
        m += p
        while len(m) % 256:
            m.append(FALSE)
    assert len(m) == 39 * 256
    out = sha256(cs, m)
    le = []
    for k in range(0, 256, 8):
        le += list(reversed(out[k:k + 8]))
    return pack_bits(cs, le)


# ------------------------------------------------------------------------------------------ the stacked circuit
BASE_DEGREE, EXP_DEGREE = 6, 8


def stacked_circuit(cs, inst, layers, nodes, shape):
    """StackedCircuit::synthesize (circuit/proof.hpp:98-165) + Proof::synthesize (circuit/params.hpp:93-238)
    for one partition.  inst: dict with replica_id, comm_d, comm_r, comm_r_last, comm_c (ints) and
    challenges: list of dicts {index, data_leaf, d_siblings, r_siblings, c_column, c_siblings,
    drg: [(index, column, siblings)] x 6, exp: [...] x 8}.  Tree D is binary SHA-256 over `nodes`; trees C
    and R-last have `shape` = (base, sub, top) Poseidon arities."""
    rid = cs.alloc(inst["replica_id"])
    inputize(cs, rid)
    rid_bits = reverse_bit_numbering(to_bits_le(cs, rid))
    comm_d = cs.alloc(inst["comm_d"])
    inputize(cs, comm_d)
    comm_r = cs.alloc(inst["comm_r"])
    inputize(cs, comm_r)
    comm_r_last = cs.alloc(inst["comm_r_last"])
    comm_c = cs.alloc(inst["comm_c"])
    h = poseidon_hash_circuit(cs, [comm_c, comm_r_last], 2)
    equal(cs, comm_r, h)
    d_levels = tree_levels(nodes, (2, 0, 0))
    c_levels = tree_levels(nodes, shape)
    for ch in inst["challenges"]:
        challenge_synthesize(cs, ch, layers, comm_d, comm_c, comm_r_last, rid_bits, d_levels, c_levels)
    return cs


def challenge_synthesize(cs, ch, layers, comm_d, comm_c, comm_r_last, rid_bits, d_levels, c_levels):
    data_leaf = cs.alloc(ch["data_leaf"])
    por_synthesize(cs, data_leaf, ch["index"], [[s] for s in ch["d_siblings"]], comm_d, d_levels, "sha256")
    cols = {}
    for kind in ("drg", "exp"):
        cols[kind] = []
        for idx, column, sibs in ch[kind]:
            assert len(column) == layers
            col = [cs.alloc(v) for v in column]  # ColumnProof::alloc: the column's values
            val = poseidon_hash_circuit(cs, col, layers)  # column hash (hash_single_column)
            por_synthesize(cs, val, idx, sibs, comm_c, c_levels, "poseidon")
            cols[kind].append(col)
    chal_bits = uint64_alloc(cs, ch["index"])
    pack_into_inputs(cs, chal_bits)
    labels = []
    for layer in range(1, layers + 1):
        parents = [reverse_bit_numbering(to_bits_le(cs, col[layer - 1])) for col in cols["drg"]]
        if layer > 1:
            parents += [reverse_bit_numbering(to_bits_le(cs, col[layer - 2])) for col in cols["exp"]]
            exp = parents + parents + parents[:9]
        else:
            exp = parents * 6 + parents[:1]
        labels.append(create_label_circuit(cs, rid_bits, exp, layer, chal_bits))
    # encoding: key = the last label, encoded node = key + data (gadgets/encode.rs -> constraint::add)
    enc = add(cs, labels[-1], data_leaf)
    por_synthesize(cs, enc, ch["index"], ch["r_siblings"], comm_r_last, c_levels, "poseidon")
    # the challenged column's hash over the labels just recomputed, included in tree C
    col_hash = poseidon_hash_circuit(cs, labels, layers)
    por_synthesize(cs, col_hash, ch["index"], ch["c_siblings"], comm_c, c_levels, "poseidon")


# ------------------------------------------------------------------------------------------ Fallback PoSt
def fallback_post_circuit(cs, inst, shape):
    """FallbackPoStCircuit::synthesize over a partition's sectors (the reference carries the data,
    post/fallback/circuit.hpp:38-86; the body restated here is rust-fil-proofs storage-proofs-post
    fallback/circuit.rs Sector::synthesize): comm_c, comm_r_last and comm_r allocated in that order, comm_r
    inputized, hash2(comm_c, comm_r_last) == comm_r, then one private PoR per challenge whose root is the
    allocated comm_r_last.  Pinned by the reference's partition sizes (constants.hpp:85-89): 2349 sectors x 10
    challenges over 2^30-node 8-8-0 trees = 125,279,217 constraints (tests/test_cpu_post_circuit.py)."""
    levels = tree_levels(inst["nodes"], shape)
    for sec in inst["sectors"]:
        comm_c = cs.alloc(sec["comm_c"])
        comm_r_last = cs.alloc(sec["comm_r_last"])
        comm_r = cs.alloc(sec["comm_r"])
        inputize(cs, comm_r)
        h = poseidon_hash_circuit(cs, [comm_c, comm_r_last], 2)
        equal(cs, comm_r, h)
        for ch in sec["challenges"]:
            leaf = cs.alloc(ch["leaf"])
            por_synthesize(cs, leaf, ch["index"], ch["siblings"], comm_r_last, levels, "poseidon")
    return cs


def post_constraints(sectors, challenges, levels):
    """closed form of fallback_post_circuit's size: per sector 1 (comm_r input) + 311 (Poseidon-2) + 1
    (equality), per challenge sum over levels of (index bits + insert + Poseidon) + 1 (path input) + 1 (root)"""
    ins = {2: 2, 4: 8, 8: 22}
    nb = {2: 1, 4: 2, 8: 3}
    por = sum(nb[a] + ins[a] + poseidon_constraints(a) for a in levels) + 2
    return sectors * (1 + poseidon_constraints(2) + 1 + challenges * por)
