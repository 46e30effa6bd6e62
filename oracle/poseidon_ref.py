"""poseidon_ref.py -- TEST INFRASTRUCTURE ONLY: plain-integer restatement of the Poseidon hash over the
BLS12-381 scalar field that Filecoin's tree C / tree R-last use.

PARITY UNPINNED.  The reference calls crypto3's hash (`crypto3::hashes::poseidon<FieldType, 2, 2>` and
`<FieldType, 11, 11>`: libs/storage/include/nil/filecoin/storage/proofs/porep/stacked/vanilla/hash.hpp:
37-47) for column hashing and an arity-8 Poseidon Merkle tree for tree C / tree R-last
(porep/stacked/vanilla/proof.hpp:383-810, ColumnTreeBuilder<ColumnArity, TreeArity>, TreeBuilder<8>).
The crypto3 hash submodule is empty in /root/reference (.gitmodules; no pinned commit) and the tree
holds no Poseidon test vector, so this file restates the published construction Filecoin's
implementation (filecoin-project/neptune, the Rust library the reference's `ColumnTreeBuilder` /
`TreeBuilder` / `BatcherType::GPU` names come from) follows, with every choice stated:

  * field: Fr of BLS12-381, r = 0x73eda753...00000001, 255 bits; S-box x^5.
  * width t = arity + 1; state = [domain tag, x_1 .. x_arity]; the digest is state[1] after the
    permutation.  Merkle-tree hashing (tree C columns and tree nodes) uses the tag 2^arity - 1.
  * rounds: R_F = 8 full (4 + 4) around R_P partial rounds, R_P = 55 / 56 / 57 / 57 / 59 for
    arity 2 / 4 / 8 / 11 / 16 ("Standard" strength).
  * round: add the t round constants of the round, S-box (all elements in a full round, element 0 in a
    partial round), multiply by the MDS matrix (state' = state * M; M is symmetric).
  * MDS: Cauchy matrix M[i][j] = 1 / (x_i + y_j) with x_i = i, y_j = t + j.
  * round constants: the Poseidon reference's Grain LFSR -- 80-bit state seeded with the bits of
    (field = 1: 2 bits, sbox = SBOX_FIELD: 4 bits, field size 255: 12 bits, t: 12 bits, R_F: 10 bits,
    R_P: 10 bits, thirty 1 bits), update b_80 = b_62 ^ b_51 ^ b_38 ^ b_23 ^ b_13 ^ b_0, 160 warm-up
    bits discarded, self-shrinking output (a pair (b1, b2) emits b2 iff b1 = 1), 255 output bits per
    candidate read most-significant first, candidates >= r rejected; (R_F + R_P) * t constants, used
    in order, t per round.
    SBOX_FIELD = 1 is the value Filecoin's implementation seeds the LFSR with (an assumption of this
    restatement, kept as a parameter).

The GPU kernel evaluates the same permutation in the sparse-matrix form (round constants of the partial
rounds folded forward, M factored per partial round); this file evaluates it literally, so the two
agree only if both are right.
"""

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
FIELD_BITS = 255
SBOX_FIELD = 1
ROUNDS = {2: (8, 55), 4: (8, 56), 8: (8, 57), 11: (8, 57), 16: (8, 59)}


def _grain_bits(t, r_f, r_p, field=1, sbox=SBOX_FIELD, field_size=FIELD_BITS):
    seed = []

    def app(n, v):
        seed.extend((v >> i) & 1 for i in reversed(range(n)))

    app(2, field)
    app(4, sbox)
    app(12, field_size)
    app(12, t)
    app(10, r_f)
    app(10, r_p)
    app(30, (1 << 30) - 1)
    state = list(seed)
    assert len(state) == 80

    def step():
        b = state[62] ^ state[51] ^ state[38] ^ state[23] ^ state[13] ^ state[0]
        state.pop(0)
        state.append(b)
        return b

    for _ in range(160):
        step()
    while True:
        b1 = step()
        b2 = step()
        if b1:
            yield b2


def round_constants(arity):
    t = arity + 1
    r_f, r_p = ROUNDS[arity]
    gen = _grain_bits(t, r_f, r_p)
    out = []
    while len(out) < (r_f + r_p) * t:
        v = 0
        for _ in range(FIELD_BITS):
            v = (v << 1) | next(gen)
        if v < R:
            out.append(v)
    return out


def mds(arity):
    t = arity + 1
    return [[pow(i + t + j, R - 2, R) for j in range(t)] for i in range(t)]


class Poseidon:
    def __init__(self, arity):
        self.arity = arity
        self.t = arity + 1
        self.r_f, self.r_p = ROUNDS[arity]
        self.rc = round_constants(arity)
        self.m = mds(arity)
        self.tag = (1 << arity) - 1

    def permute(self, state):
        t, m, rc = self.t, self.m, self.rc
        s = [x % R for x in state]
        k = 0
        half = self.r_f // 2
        for rnd in range(self.r_f + self.r_p):
            s = [(s[i] + rc[k + i]) % R for i in range(t)]
            k += t
            full = rnd < half or rnd >= half + self.r_p
            if full:
                s = [pow(x, 5, R) for x in s]
            else:
                s[0] = pow(s[0], 5, R)
            s = [sum(s[i] * m[i][j] for i in range(t)) % R for j in range(t)]
        return s

    def hash(self, xs):
        assert len(xs) == self.arity
        return self.permute([self.tag] + list(xs))[1]


def _mat_inv(a):
    """Gauss-Jordan inverse over Fr (plain ints)."""
    n = len(a)
    m = [list(row) + [1 if i == j else 0 for j in range(n)] for i, row in enumerate(a)]
    for c in range(n):
        p = next(r for r in range(c, n) if m[r][c] % R)
        m[c], m[p] = m[p], m[c]
        iv = pow(m[c][c], R - 2, R)
        m[c] = [x * iv % R for x in m[c]]
        for r in range(n):
            if r != c and m[r][c]:
                f = m[r][c]
                m[r] = [(x - f * y) % R for x, y in zip(m[r], m[c])]
    return [row[n:] for row in m]


def _mat_mul(a, b):
    return [[sum(a[i][k] * b[k][j] for k in range(len(b))) % R for j in range(len(b[0]))] for i in range(len(a))]


def sparse_form(arity):
    """The optimised evaluation (Poseidon paper, appendix B; neptune's "optimized static" constants), derived
    here independently of the library's C++: round constants of elements 1.. of every partial round folded
    into the next round; M A_{k-1} = A_k B_k with A_k = diag(1, M^^k), B_k = [[m00, v^T M^^{k-1}],
    [M^^-k w, I]]; the last partial round uses the dense M A_{R_P - 1}.  Returns (rc_first, rc_part, rc_last,
    sparse rows [(row, w_hat)], dense)."""
    h = poseidon(arity)
    t, rf, rp, m = h.t, h.r_f, h.r_p, h.m
    rc = [h.rc[r * t:(r + 1) * t] for r in range(rf + rp)]
    half = rf // 2
    for r in range(half, half + rp):
        tail = [0] + rc[r][1:]
        add = [sum(m[i][j] * tail[j] for j in range(t)) % R for i in range(t)]
        rc[r + 1] = [(x + y) % R for x, y in zip(rc[r + 1], add)]
        rc[r] = [rc[r][0]] + [0] * (t - 1)
    mh = [row[1:] for row in m[1:]]
    v, w = m[0][1:], [m[i][0] for i in range(1, t)]
    mh_inv = _mat_inv(mh)
    ah = [[1 if i == j else 0 for j in range(t - 1)] for i in range(t - 1)]
    w_k = w
    rows = []
    for _ in range(1, rp):
        row = [m[0][0]] + [sum(v[q] * ah[q][j] for q in range(t - 1)) % R for j in range(t - 1)]
        ah = _mat_mul(mh, ah)
        w_k = [sum(mh_inv[i][q] * w_k[q] for q in range(t - 1)) % R for i in range(t - 1)]
        rows.append((row, list(w_k)))
    a = [[1 if (i == 0 and j == 0) else 0 for j in range(t)] for i in range(t)]
    for i in range(t - 1):
        for j in range(t - 1):
            a[i + 1][j + 1] = ah[i][j]
    dense = _mat_mul(m, a)
    return rc[:half], [rc[r][0] for r in range(half, half + rp)], rc[half + rp:], rows, dense


def permute_sparse(arity, state):
    """The permutation evaluated in the sparse form (must equal Poseidon.permute)."""
    h = poseidon(arity)
    t = h.t
    first, part, last, rows, dense = sparse_form(arity)
    s = [x % R for x in state]

    def full(s, c):
        s = [pow((x + y) % R, 5, R) for x, y in zip(s, c)]
        return [sum(h.m[i][j] * s[j] for j in range(t)) % R for i in range(t)]

    for c in first:
        s = full(s, c)
    for k, (row, wh) in enumerate(rows):
        s[0] = pow((s[0] + part[k]) % R, 5, R)
        n0 = sum(a * b for a, b in zip(row, s)) % R
        s = [n0] + [(s[j + 1] + wh[j] * s[0]) % R for j in range(t - 1)]
    s[0] = pow((s[0] + part[-1]) % R, 5, R)
    s = [sum(dense[i][j] * s[j] for j in range(t)) % R for i in range(t)]
    for c in last:
        s = full(s, c)
    return s


_CACHE = {}


def poseidon(arity):
    if arity not in _CACHE:
        _CACHE[arity] = Poseidon(arity)
    return _CACHE[arity]


def fr_from_bytes(b):
    v = int.from_bytes(b, "little")
    assert v < R
    return v


def fr_to_bytes(v):
    return int(v).to_bytes(32, "little")


def hash_columns(layers):
    """tree C leaves: one arity-len(layers) hash per node over (layer_1[j], ..., layer_L[j])."""
    h = poseidon(len(layers))
    return [h.hash([layer[j] for layer in layers]) for j in range(len(layers[0]))]


def merkle_rows(leaves, arity):
    """All rows of the arity-`arity` Poseidon Merkle tree, base row first, root row last."""
    h = poseidon(arity)
    rows = [list(leaves)]
    while len(rows[-1]) > 1:
        cur = rows[-1]
        assert len(cur) % arity == 0
        rows.append([h.hash(cur[i:i + arity]) for i in range(0, len(cur), arity)])
    return rows


def tree_data(leaves, arity, rows_to_discard=0):
    """The cached tree rows: every row above the base except the `rows_to_discard` lowest of them
    (neptune TreeBuilder::tree_size / merkletree get_merkle_tree_cache_size semantics), flattened."""
    rows = merkle_rows(leaves, arity)
    out = []
    for r in rows[1 + rows_to_discard:]:
        out.extend(r)
    return out


def encode(key, data):
    """Replica node = label + data node in Fr (porep encode, vanilla/proof.hpp generate_tree_r_last)."""
    return (key + data) % R
