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
