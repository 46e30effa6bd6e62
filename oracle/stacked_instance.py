"""stacked_instance.py -- TEST INFRASTRUCTURE ONLY: small, fully built stacked-PoRep instances (a replica with
real trees) whose vanilla openings satisfy the stacked circuit, and the reference's public-input order; the
same for Fallback PoSt partitions (generate_post: sectors with full trees R-last, challenges derived by
generate_leaf_challenge, post/fallback/vanilla.hpp:398-411).

  * tree D: binary SHA-256 tree over the data nodes (node hash = sha256(left LE || right LE) with byte 31 &=
    0x3f; pinned by the reference's compute_comm_d vectors, tests/test_cpu_sdr.py);
  * labels: random for every (layer, node) except the challenged nodes, whose labels are recomputed from
    their parents' columns exactly as create_label hashes them (replica_id | layer u32 BE | node u64 BE |
    zeros | 37 parents; vanilla/create_label.hpp:76-77, params.hpp:199-212 for the 6 x 6 + 1 / 14 x 2 + 9
    expansion), so the labelling check holds while the graph itself is synthetic (the circuit takes the
    parents' indices as public inputs, it does not recompute the graph);
  * tree C: Poseidon column hashes (arity = layers) under a (base, sub, top) Poseidon tree; tree R-last: the
    encoded nodes data + last label under the same shape; comm_r = Poseidon-2(comm_c, comm_r_last)
    (StackedCircuit: H(comm_c || comm_r_last), circuit/proof.hpp:98-165);
  * generate_public_inputs (circuit/proof.hpp:186-269 / rust-fil-proofs StackedCompound): replica_id, comm_d,
    comm_r, then per challenge the packed path index of tree D, of the 6 DRG and 8 expander parents in tree C,
    the challenge (UInt64), its tree R-last and tree C paths.  A private PoR's only input is the packed path
    index, i.e. the leaf index itself.
"""
import hashlib
import random

from poseidon_ref import R, Poseidon

BASE_DEGREE, EXP_DEGREE = 6, 8
_P = {}


def poseidon(arity, xs):
    if arity not in _P:
        _P[arity] = Poseidon(arity)
    return _P[arity].hash(xs)


def sha_node(a, b):
    d = bytearray(hashlib.sha256(a.to_bytes(32, "little") + b.to_bytes(32, "little")).digest())
    d[31] &= 0x3F
    return int.from_bytes(d, "little")


def create_label(replica_id, layer, node, parents37):
    msg = replica_id.to_bytes(32, "little") + layer.to_bytes(4, "big") + node.to_bytes(8, "big") + bytes(20)
    msg += b"".join(p.to_bytes(32, "little") for p in parents37)
    d = bytearray(hashlib.sha256(msg).digest())
    d[31] &= 0x3F
    return int.from_bytes(d, "little")


def expand_parents(parents, layer):
    """params.hpp:199-212: layer 1 has 6 DRG parents -> 6 x 6 + 1; later layers 14 -> 14 x 2 + 9"""
    return parents * 6 + parents[:1] if layer == 1 else parents + parents + parents[:9]


def build_tree(leaves, shape, hasher):
    """rows bottom-up; each row a list.  shape = (base, sub, top) arities (0 = absent)"""
    base, sub, top = shape
    n_base = (sub or 1) * (top or 1)
    per = len(leaves) // n_base
    arities = []
    m = per
    while m > 1:
        arities.append(base)
        m //= base
    if sub:
        arities.append(sub)
    if top:
        arities.append(top)
    rows = [list(leaves)]
    for a in arities:
        cur = rows[-1]
        rows.append([hasher(a, cur[i:i + a]) for i in range(0, len(cur), a)])
    return rows, arities


def siblings(rows, arities, index):
    out, j = [], index
    for lvl, a in enumerate(arities):
        g = j // a
        grp = rows[lvl][g * a:(g + 1) * a]
        out.append([v for k, v in enumerate(grp) if k != j % a])
        j = g
    return out


def generate(nodes, layers, shape, n_challenges, seed=1):
    rng = random.Random(seed)
    fr = lambda: rng.randrange(R)
    replica_id = fr()
    data = [fr() for _ in range(nodes)]
    labels = [[fr() >> 2 for _ in range(nodes)] for _ in range(layers)]  # labels are 254-bit values
    challenges = rng.sample(range(nodes), n_challenges)
    others = [i for i in range(nodes) if i not in challenges]
    graph = {}
    for c in challenges:
        drg = [rng.choice(others) for _ in range(BASE_DEGREE)]
        exp = [rng.choice(others) for _ in range(EXP_DEGREE)]
        graph[c] = (drg, exp)
        for layer in range(1, layers + 1):
            ps = [labels[layer - 1][p] for p in drg]
            if layer > 1:
                ps += [labels[layer - 2][p] for p in exp]
            labels[layer - 1][c] = create_label(replica_id, layer, c, expand_parents(ps, layer))
    d_rows, d_ar = build_tree(data, (2, 0, 0), lambda a, xs: sha_node(*xs))
    ph = lambda a, xs: poseidon(a, xs)
    col_hash = [poseidon(layers, [labels[l][i] for l in range(layers)]) for i in range(nodes)]
    c_rows, c_ar = build_tree(col_hash, shape, ph)
    enc = [(data[i] + labels[layers - 1][i]) % R for i in range(nodes)]
    r_rows, r_ar = build_tree(enc, shape, ph)
    comm_d, comm_c, comm_r_last = d_rows[-1][0], c_rows[-1][0], r_rows[-1][0]
    comm_r = poseidon(2, [comm_c, comm_r_last])
    chs = []
    for c in challenges:
        drg, exp = graph[c]
        col = lambda i: [labels[l][i] for l in range(layers)]
        chs.append({
            "index": c,
            "data_leaf": data[c],
            "d_siblings": [s[0] for s in siblings(d_rows, d_ar, c)],
            "r_siblings": siblings(r_rows, r_ar, c),
            "c_column": col(c),
            "c_siblings": siblings(c_rows, c_ar, c),
            "drg": [(p, col(p), siblings(c_rows, c_ar, p)) for p in drg],
            "exp": [(p, col(p), siblings(c_rows, c_ar, p)) for p in exp],
        })
    return {"replica_id": replica_id, "comm_d": comm_d, "comm_c": comm_c, "comm_r_last": comm_r_last,
            "comm_r": comm_r, "challenges": chs, "nodes": nodes, "layers": layers, "shape": shape}


def public_inputs(inst):
    """generate_public_inputs order (without ONE)"""
    out = [inst["replica_id"], inst["comm_d"], inst["comm_r"]]
    for ch in inst["challenges"]:
        c = ch["index"]
        out.append(c)  # tree D path (private PoR: the packed index bits)
        out += [p for p, _, _ in ch["drg"]]
        out += [p for p, _, _ in ch["exp"]]
        out += [c, c, c]  # the challenge (UInt64), tree R-last path, tree C path
    return out


# ------------------------------------------------------------------------------------------ Fallback PoSt
def generate_leaf_challenge(randomness, sector_id, leaf_challenge_index, nodes):
    """post/fallback/vanilla.hpp:398-411"""
    h = hashlib.sha256(randomness.to_bytes(32, "little") + sector_id.to_bytes(8, "little") +
                       leaf_challenge_index.to_bytes(8, "little")).digest()
    return int.from_bytes(h[:8], "little") % nodes


def generate_post(n_sectors, challenges, nodes, shape, seed=1, partition=0):
    """A Fallback PoSt partition over fully built trees R-last: per sector random leaves (the encoded replica
    nodes), the (base, sub, top) Poseidon tree, a random comm_c, comm_r = Poseidon-2(comm_c, comm_r_last); the
    challenged leaves of sector i are generate_leaf_challenge(randomness, id, (partition * S + i) * C + n)
    (prove_all_partitions, vanilla.hpp:222-236)."""
    rng = random.Random(seed)
    fr = lambda: rng.randrange(R)
    randomness = fr()
    sectors = []
    for i in range(n_sectors):
        sid = rng.randrange(2 ** 40)
        leaves = [fr() for _ in range(nodes)]
        rows, ar = build_tree(leaves, shape, lambda a, xs: poseidon(a, xs))
        comm_r_last, comm_c = rows[-1][0], fr()
        chs = []
        for n in range(challenges):
            idx = generate_leaf_challenge(randomness, sid, (partition * n_sectors + i) * challenges + n, nodes)
            chs.append({"index": idx, "leaf": leaves[idx], "siblings": siblings(rows, ar, idx)})
        sectors.append({"id": sid, "comm_c": comm_c, "comm_r_last": comm_r_last,
                        "comm_r": poseidon(2, [comm_c, comm_r_last]), "challenges": chs})
    return {"randomness": randomness, "sectors": sectors, "nodes": nodes, "shape": shape}


def post_public_inputs(inst):
    """FallbackPoStCompound::generate_public_inputs (without ONE): per sector comm_r, then per challenge the
    private PoR's packed path = the challenged leaf index"""
    out = []
    for sec in inst["sectors"]:
        out.append(sec["comm_r"])
        out += [ch["index"] for ch in sec["challenges"]]
    return out


def winning_post_setup_params(challenge_count=66, sector_count=1):
    """proofs/parameters.hpp:58-68 (constants.hpp:54-55: 66 challenges, 1 sector) -> (param_sector_count,
    param_challenge_count)"""
    assert challenge_count % sector_count == 0, "sector count must divide challenge count"
    ps = challenge_count // sector_count
    pc = challenge_count // ps
    assert ps * pc == challenge_count, "invalid parameters calculated"
    return ps, pc


def generate_winning_post(nodes, shape, seed=1, challenge_count=66, sector_count=1):
    """A Winning-PoSt partition over fully built trees R-last, as generate_winning_post lays it out
    (api/post.hpp:190-230): the sector_count replicas (random leaves, the (base, sub, top) Poseidon tree, random
    comm_c) repeated over param_sector_count circuit sectors; circuit sector i, challenge n opens
    generate_leaf_challenge(randomness, id, i * param_challenge_count + n) (prove_all_partitions,
    vanilla.hpp:222-236, one partition)."""
    ps, pc = winning_post_setup_params(challenge_count, sector_count)
    rng = random.Random(seed)
    fr = lambda: rng.randrange(R)
    randomness = fr()
    reps = []
    for _ in range(sector_count):
        sid = rng.randrange(2 ** 40)
        leaves = [fr() for _ in range(nodes)]
        rows, ar = build_tree(leaves, shape, lambda a, xs: poseidon(a, xs))
        comm_c = fr()
        reps.append((sid, leaves, rows, ar, comm_c))
    sectors = []
    for i in range(ps):
        for sid, leaves, rows, ar, comm_c in reps:
            k = len(sectors)
            chs = []
            for n in range(pc):
                idx = generate_leaf_challenge(randomness, sid, k * pc + n, nodes)
                chs.append({"index": idx, "leaf": leaves[idx], "siblings": siblings(rows, ar, idx)})
            comm_r_last = rows[-1][0]
            sectors.append({"id": sid, "comm_c": comm_c, "comm_r_last": comm_r_last,
                            "comm_r": poseidon(2, [comm_c, comm_r_last]), "challenges": chs})
    return {"randomness": randomness, "sectors": sectors, "nodes": nodes, "shape": shape}
