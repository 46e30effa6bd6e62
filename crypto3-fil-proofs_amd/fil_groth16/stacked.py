"""Stacked-PoRep and Fallback-PoSt circuits: R1CS shape and GPU witness generation.

Mirrors the synthesis half of the reference's compound proofs:
  StackedCircuit                  StackedCompound::circuit + StackedCircuit::synthesize
                                  (libs/storage/include/nil/filecoin/storage/proofs/porep/stacked/circuit/
                                  proof.hpp:98-165; Proof::synthesize, params.hpp:93-238)
  StackedCircuit.public_inputs    generate_public_inputs (circuit/proof.hpp:186-269)
  instance_slots                  the circuit Proof built from a vanilla proof (params.hpp:69-90): the openings
                                  the gadgets consume, in the library's slot layout
  FallbackPoStCircuit             FallbackPoStCircuit / Sector (post/fallback/circuit.hpp:38-86; the synthesize
                                  body is rust-fil-proofs storage-proofs-post fallback/circuit.rs): Window and
                                  Winning PoSt partitions
  winning_post_setup_params       proofs/parameters.hpp:58-68: Winning PoSt's 66 challenges over 1 sector become
                                  66 circuit sectors x 1 challenge (WinningPoStCircuit)
  winning_post_sectors            generate_winning_post's replica repetition (api/post.hpp:205-218)
  generate_leaf_challenge         post/fallback/vanilla.hpp:398-411
  post_slots                      a partition's sector proofs (vanilla.hpp:188-251) in the slot layout
The R1CS is built on the host once per shape (mi_stacked_build / mi_post_build; the blank circuit), the
witness of every partition on the GPU (mi_stacked_witness*).  There is no CPU witness path.
"""
import ctypes

import numpy as np

from ._lib import check, lib, torch_sync
from .core import FR_MODULUS, Circuit, _R1CS


class _Shape(ctypes.Structure):
    _fields_ = [("layers", ctypes.c_uint32), ("challenges", ctypes.c_uint32), ("nodes", ctypes.c_uint64),
                ("base_arity", ctypes.c_uint32), ("sub_arity", ctypes.c_uint32), ("top_arity", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


INFO_KEYS = ("constraints", "inputs", "aux", "slots", "stride", "depth_d", "path_c", "ops", "levels", "sha_blocks",
             "poseidon_hashes", "r1cs_entries")


def tree_arities(nodes, base, sub=0, top=0):
    """tree C / tree R-last level arities, leaf upward (rust-fil-proofs base / sub / top trees)"""
    per = nodes // ((sub or 1) * (top or 1))
    out = []
    while per > 1:
        out.append(base)
        per //= base
    return out + [a for a in (sub, top) if a]


class _PostShape(ctypes.Structure):
    _fields_ = [("sectors", ctypes.c_uint32), ("challenges", ctypes.c_uint32), ("nodes", ctypes.c_uint64),
                ("base_arity", ctypes.c_uint32), ("sub_arity", ctypes.c_uint32), ("top_arity", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


class _BuiltCircuit:
    """A circuit built by the library (R1CS + GPU witness program); subclasses name the shape."""

    def _finish(self, with_r1cs):
        out = (ctypes.c_uint64 * len(INFO_KEYS))()
        check(lib().mi_stacked_info(self.h, out))
        self.info = dict(zip(INFO_KEYS, list(out)))
        self.with_r1cs = with_r1cs

    @property
    def num_constraints(self):
        return self.info["constraints"]

    @property
    def num_inputs(self):
        return self.info["inputs"]

    @property
    def num_aux(self):
        return self.info["aux"]

    @property
    def num_vars(self):
        return self.num_inputs + self.num_aux

    def csr(self):
        """numpy views (valid while this object lives): 3 x (row_ptr u64, col u32, coeff u8[nnz * 32])"""
        s = _R1CS()
        check(lib().mi_stacked_r1cs(self.h, ctypes.byref(s)))
        n = s.num_constraints
        mats = []
        for m in range(3):
            rp = np.ctypeslib.as_array((ctypes.c_uint64 * (n + 1)).from_address(s.row_ptr[m]))
            nnz = int(rp[-1])
            col = (np.ctypeslib.as_array((ctypes.c_uint32 * nnz).from_address(s.col[m])) if nnz
                   else np.zeros(0, np.uint32))
            co = (np.ctypeslib.as_array((ctypes.c_uint8 * (32 * nnz)).from_address(s.coeff[m])) if nnz
                  else np.zeros(0, np.uint8))
            mats.append((rp, col, co))
        return mats

    def load(self, ctx) -> Circuit:
        """the circuit on the device, uploaded from the builder's compact form (mi_stacked_load)"""
        h = ctypes.c_void_p()
        check(lib().mi_stacked_load(ctx.h, self.h, ctypes.byref(h)))
        return Circuit.from_handle(ctx, h)

    def public_inputs(self, slots: bytes) -> bytes:
        out = ctypes.create_string_buffer(32 * (self.num_inputs - 1))
        check(lib().mi_stacked_public_inputs(self.h, bytes(slots), out))
        return out.raw

    def witness(self, ctx, slots: bytes) -> bytes:
        """z = ONE ++ inputs ++ aux (32 B each), computed on the GPU, returned to the host"""
        out = ctypes.create_string_buffer(32 * self.num_vars)
        check(lib().mi_stacked_witness(ctx.h, self.h, bytes(slots), out))
        return out.raw

    def witness_dev(self, ctx, slots_dev_ptr: int, z_dev_ptr: int):
        torch_sync(ctx)
        check(lib().mi_stacked_witness_dev(ctx.h, self.h, ctypes.c_void_p(slots_dev_ptr), ctypes.c_void_p(z_dev_ptr)))

    def __del__(self):
        try:
            lib().mi_stacked_free(self.h)
        except Exception:
            pass


class StackedCircuit(_BuiltCircuit):
    """One partition's circuit of a shape: layers (2 or 11), challenges, nodes, tree C / R-last arities."""

    def __init__(self, layers=2, challenges=1, nodes=8, base=8, sub=0, top=0, with_r1cs=True):
        sh = _Shape(layers, challenges, nodes, base, sub, top, 0)
        self.h = ctypes.c_void_p()
        check(lib().mi_stacked_build(ctypes.byref(sh), int(with_r1cs), ctypes.byref(self.h)))
        self.layers, self.challenges, self.nodes = layers, challenges, nodes
        self.arities = tree_arities(nodes, base, sub, top)
        self._finish(with_r1cs)


class FallbackPoStCircuit(_BuiltCircuit):
    """One Fallback PoSt partition: `sectors` sectors x `challenges` private tree R-last inclusion proofs
    (Window PoSt at 32 GiB: 2349 x 10 over 2^30-node 8-8-0 trees = 125,279,217 constraints, constants.hpp:85-89;
    Winning PoSt: 66 sectors x 1 challenge, WinningPoStCircuit)."""

    def __init__(self, sectors=1, challenges=1, nodes=64, base=8, sub=0, top=0, with_r1cs=True):
        sh = _PostShape(sectors, challenges, nodes, base, sub, top, 0)
        self.h = ctypes.c_void_p()
        check(lib().mi_post_build(ctypes.byref(sh), int(with_r1cs), ctypes.byref(self.h)))
        self.sectors, self.challenges, self.nodes = sectors, challenges, nodes
        self.arities = tree_arities(nodes, base, sub, top)
        self._finish(with_r1cs)


WINNING_POST_CHALLENGE_COUNT = 66  # constants.hpp:54
WINNING_POST_SECTOR_COUNT = 1  # constants.hpp:55


def winning_post_setup_params(challenge_count: int = WINNING_POST_CHALLENGE_COUNT,
                              sector_count: int = WINNING_POST_SECTOR_COUNT):
    """proofs/parameters.hpp:58-68 winning_post_setup_params -> (param_sector_count, param_challenge_count):
    the post_config's challenges over its sectors become challenge_count / sector_count circuit sectors of
    challenge_count / param_sector_count challenges each (66 / 1 -> 66 sectors x 1 challenge)."""
    if sector_count <= 0 or challenge_count <= 0 or challenge_count % sector_count:
        raise ValueError("sector count must divide challenge count")
    param_sector_count = challenge_count // sector_count
    param_challenge_count = challenge_count // param_sector_count
    if param_sector_count * param_challenge_count != challenge_count:
        raise ValueError("invalid parameters calculated")
    return param_sector_count, param_challenge_count


class WinningPoStCircuit(FallbackPoStCircuit):
    """The Winning PoSt circuit: FallbackPoSt set up with winning_post_setup_params (parameters.hpp:58-68), one
    partition (partitions unset, api/post.hpp:193).  At 32 GiB (2^30-node 8-8-0 trees R-last): 66 sectors x 1
    challenge = 370,590 constraints, 1 + 66 x 2 = 133 public inputs, domain 2^19."""

    def __init__(self, nodes, base=8, sub=8, top=0, challenge_count=WINNING_POST_CHALLENGE_COUNT,
                 sector_count=WINNING_POST_SECTOR_COUNT, with_r1cs=True):
        ps, pc = winning_post_setup_params(challenge_count, sector_count)
        super().__init__(ps, pc, nodes, base, sub, top, with_r1cs)
        self.replicas = sector_count


def winning_post_sectors(replicas, param_sector_count: int):
    """api/post.hpp:205-218: for i in 0..param_sector_count, for each replica (in sector-id order): one
    public/private sector -- the post_config's replicas repeated param_sector_count times (66 copies of the one
    Winning-PoSt replica).  The reference's C++ sizes its vectors and then pushes behind them; the sector list
    it means (rust-fil-proofs winning_post.rs) is this one."""
    return [r for _ in range(param_sector_count) for r in replicas]


def generate_leaf_challenge(randomness: int, sector_id: int, leaf_challenge_index: int, nodes: int) -> int:
    """post/fallback/vanilla.hpp:398-411: SHA-256(randomness (32 B LE) || sector_id u64 LE || index u64 LE),
    the first 8 bytes as a little-endian u64, mod the sector's node count"""
    import hashlib

    h = hashlib.sha256(int(randomness).to_bytes(32, "little") + int(sector_id).to_bytes(8, "little") +
                       int(leaf_challenge_index).to_bytes(8, "little")).digest()
    return int.from_bytes(h[:8], "little") % nodes


def post_challenges(randomness: int, sector_ids, challenges: int, nodes: int, partition: int = 0,
                    sectors_per_partition: int = None):
    """the challenged leaves of one partition's sectors (prove_all_partitions, vanilla.hpp:222-236): sector i of
    partition j, challenge n -> generate_leaf_challenge(randomness, id, (j * sectors + i) * challenges + n)"""
    per = sectors_per_partition or len(sector_ids)
    return [[generate_leaf_challenge(randomness, sid, (partition * per + i) * challenges + n, nodes)
             for n in range(challenges)] for i, sid in enumerate(sector_ids)]


def post_slots(circuit: FallbackPoStCircuit, sectors) -> bytes:
    """Pack a partition's sector proofs into the slot layout (mi355x_groth16.h, mi_post_build).  sectors: one
    dict per sector with comm_r, comm_c, comm_r_last and challenges: [{index, leaf, siblings}] (siblings per
    tree level, the arity - 1 other children in position order).  Fewer sectors than the circuit takes are
    padded by repeating the last one (prove_all_partitions, vanilla.hpp:241-245)."""
    if not sectors or len(sectors) > circuit.sectors:
        raise ValueError(f"1 .. {circuit.sectors} sectors per partition, got {len(sectors)}")
    sectors = list(sectors) + [sectors[-1]] * (circuit.sectors - len(sectors))
    out = []
    for sec in sectors:
        out += [_fr(sec["comm_r"]), _fr(sec["comm_c"]), _fr(sec["comm_r_last"])]
        if len(sec["challenges"]) != circuit.challenges:
            raise ValueError(f"{circuit.challenges} challenge(s) per sector, got {len(sec['challenges'])}")
        for ch in sec["challenges"]:
            if [len(s) + 1 for s in ch["siblings"]] != circuit.arities:
                raise ValueError("sibling levels do not match the tree shape")
            out += [_fr(ch["index"]), _fr(ch["leaf"])]
            out += [_fr(v) for lvl in ch["siblings"] for v in lvl]
    buf = b"".join(out)
    assert len(buf) == 32 * circuit.info["slots"]
    return buf


def synthetic_post_instance(ctx, circuit: FallbackPoStCircuit, seed: int = 1, partition: int = 0, replicas=None):
    """A consistent Fallback PoSt partition without sectors on disk (the bench's Window- and Winning-PoSt
    partitions and the GPU tests): random randomness, sector ids, comm_c and challenged leaves; challenges derived
    by generate_leaf_challenge; each replica's tree R-last built sparsely over its challenged leaves with random
    filler nodes (Poseidon on the GPU, one batched call per tree level over all replicas); comm_r =
    Poseidon-2(comm_c, comm_r_last).  replicas: distinct sectors behind the circuit's sector slots (default one
    per slot; Winning PoSt: 1, slot s holding replica s % replicas as winning_post_sectors lays them out).
    Returns (randomness, sectors in post_slots' format)."""
    from . import tree

    rng = np.random.default_rng(seed)
    S, C, nodes, ar = circuit.sectors, circuit.challenges, circuit.nodes, circuit.arities
    Q = S if replicas is None else int(replicas)
    if not 1 <= Q <= S:
        raise ValueError(f"1 .. {S} replicas behind {S} sector slots, got {Q}")

    def rand_many(k):
        b = rng.integers(0, 256, size=(k, 32), dtype=np.uint8)
        b[:, 31] &= 0x1F
        return [int.from_bytes(r.tobytes(), "little") for r in b]

    def pos_hash(a, flat):
        return tree.to_ints(tree.poseidon_hash(ctx, a, flat)) if flat else []

    randomness = rand_many(1)[0]
    ids = [int(x) for x in rng.choice(2 ** 40, size=Q, replace=False)]
    slot_ids = winning_post_sectors(ids, S // Q) + ids[:S % Q]
    chal = post_challenges(randomness, slot_ids, C, nodes, partition, S)
    levels = []  # per replica: list of {position: value} per tree level
    for q in range(Q):
        want = sorted({i for s in range(q, S, Q) for i in chal[s]})
        leaves = dict(zip(want, rand_many(len(want))))
        levels.append([leaves])
    for a in ar:  # one GPU call per level over every replica's sparse tree
        flat, parents = [], []
        for q in range(Q):
            cur = levels[q][-1]
            ps = sorted({p // a for p in cur})
            missing = [p * a + k for p in ps for k in range(a) if p * a + k not in cur]
            for m, v in zip(missing, rand_many(len(missing))):
                cur[m] = v
            for p in ps:
                flat += [cur[p * a + k] for k in range(a)]
            parents.append(ps)
        hashed = pos_hash(a, flat)
        o = 0
        for q in range(Q):
            levels[q].append(dict(zip(parents[q], hashed[o:o + len(parents[q])])))
            o += len(parents[q])
    comm_r_last = [levels[q][-1][0] for q in range(Q)]
    comm_c = rand_many(Q)
    comm_r = pos_hash(2, [v for q in range(Q) for v in (comm_c[q], comm_r_last[q])])
    sectors = []
    for s in range(S):
        q = s % Q
        chs = []
        for idx in chal[s]:
            path, j = [], idx
            for lvl, a in enumerate(ar):
                g = j // a
                path.append([levels[q][lvl][g * a + k] for k in range(a) if k != j % a])
                j = g
            chs.append({"index": idx, "leaf": levels[q][0][idx], "siblings": path})
        sectors.append({"id": ids[q], "comm_r": comm_r[q], "comm_c": comm_c[q], "comm_r_last": comm_r_last[q],
                        "challenges": chs})
    return randomness, sectors


def synthetic_winning_post_instance(ctx, circuit: WinningPoStCircuit, seed: int = 1):
    """A Winning-PoSt partition as generate_winning_post builds it (api/post.hpp:178-230): the post_config's
    replica(s) (synthetic, sparse tree R-last) repeated over the circuit's param_sector_count sector slots,
    slot i challenged at generate_leaf_challenge(randomness, id, i * challenges + n)."""
    return synthetic_post_instance(ctx, circuit, seed, 0, replicas=getattr(circuit, "replicas", 1))


def circuit_check_dev(ctx, circuit: Circuit, z_dev_ptr: int):
    """(unsatisfied rows, first unsatisfied row or None) of A z * B z = C z on the device"""
    out = (ctypes.c_uint64 * 2)()
    torch_sync(ctx)
    check(lib().mi_circuit_check_dev(ctx.h, circuit.h, ctypes.c_void_p(z_dev_ptr), out))
    return int(out[0]), (None if out[1] == 2 ** 64 - 1 else int(out[1]))


def _fr(x):
    x = int(x)
    if not 0 <= x < FR_MODULUS:
        raise ValueError("not a canonical Fr element")
    return x.to_bytes(32, "little")


def instance_slots(circuit: StackedCircuit, replica_id, comm_d, comm_r, comm_r_last, comm_c, challenges) -> bytes:
    """Pack one partition's vanilla openings into the library's slot layout (mi355x_groth16.h).  challenges: one
    dict per challenge with index, data_leaf, d_siblings (tree D, leaf upward), r_siblings / c_siblings (per
    level the arity - 1 sibling values in position order), and drg / exp: 6 / 8 tuples (index, column,
    siblings)."""
    L = circuit.layers
    out = [_fr(replica_id), _fr(comm_d), _fr(comm_r), _fr(comm_r_last), _fr(comm_c)]

    def sibs(levels):
        if [len(s) + 1 for s in levels] != circuit.arities:
            raise ValueError("sibling levels do not match the tree shape")
        return [_fr(v) for lvl in levels for v in lvl]

    if len(challenges) != circuit.challenges:
        raise ValueError(f"{circuit.challenges} challenge(s) per partition, got {len(challenges)}")
    for ch in challenges:
        out.append(_fr(ch["index"]))
        out.append(_fr(ch["data_leaf"]))
        if len(ch["d_siblings"]) != circuit.info["depth_d"]:
            raise ValueError("tree D path length")
        out += [_fr(v) for v in ch["d_siblings"]]
        out += sibs(ch["r_siblings"])
        out += sibs(ch["c_siblings"])
        if len(ch["drg"]) != 6 or len(ch["exp"]) != 8:
            raise ValueError("6 DRG and 8 expander parents per challenge")
        for idx, column, s in list(ch["drg"]) + list(ch["exp"]):
            if len(column) != L:
                raise ValueError("column length != layers")
            out.append(_fr(idx))
            out += [_fr(v) for v in column]
            out += sibs(s)
    buf = b"".join(out)
    assert len(buf) == 32 * circuit.info["slots"]
    return buf


# ---------------------------------------------------------------------------------------------- synthetic
def _sha_node(a: int, b: int) -> int:
    """tree D node hash: sha256(left LE || right LE), byte 31 &= 0x3f (compute_comm_d, pinned by the
    reference's vectors in tests/test_cpu_sdr.py)"""
    import hashlib

    d = bytearray(hashlib.sha256(a.to_bytes(32, "little") + b.to_bytes(32, "little")).digest())
    d[31] &= 0x3F
    return int.from_bytes(d, "little")


def _sparse_tree(leaves: dict, arities, hash_groups, rand):
    """Root and openings of a tree over `leaves` (position -> value) whose other nodes are random filler:
    the paths of all given leaves share one root, as in a real replica's tree.  hash_groups(arity, flat
    child values) -> parent values."""
    levels = [dict(leaves)]
    for a in arities:
        cur = levels[-1]
        parents = sorted({p // a for p in cur})
        flat = []
        for p in parents:
            for k in range(a):
                if p * a + k not in cur:
                    cur[p * a + k] = rand()
                flat.append(cur[p * a + k])
        levels.append(dict(zip(parents, hash_groups(a, flat))))
    if list(levels[-1]) != [0]:
        raise ValueError("tree shape does not reduce to one root")

    def path(idx):
        out, j = [], idx
        for lvl, a in enumerate(arities):
            g = j // a
            out.append([levels[lvl][g * a + k] for k in range(a) if k != j % a])
            j = g
        return out

    return levels[-1][0], path


def synthetic_instance(ctx, circuit: StackedCircuit, seed: int = 1):
    """A consistent instance of the circuit's shape without a sector (the bench's 32 GiB-shaped partition and
    the GPU tests): random replica id, data leaves and parent columns (6 DRG + 8 expander parents at random
    indices, none of them challenged); each challenged node's labels computed by create_label over its
    parents' columns on the GPU label kernel (sdr.create_labels: replica_id | layer | node | 37 parents);
    tree D (SHA-256), tree C (Poseidon column hashes) and tree R-last (encoded = data + last label) built
    sparsely over the opened leaves with random filler nodes, so every opening of the partition meets one
    root; comm_r = Poseidon-2(comm_c, comm_r_last).  Returns the instance in instance_slots' format."""
    from . import sdr, tree

    rng = np.random.default_rng(seed)
    L, C, nodes = circuit.layers, circuit.challenges, circuit.nodes

    def rand():
        b = bytearray(rng.bytes(32))
        b[31] &= 0x1F
        return int.from_bytes(b, "little")

    def pos_hash(a, flat):
        return tree.to_ints(tree.poseidon_hash(ctx, a, flat)) if flat else []

    if C + 14 > nodes:
        raise ValueError("too few nodes for distinct challenges and parents")
    chal = []
    while len(chal) < C:
        x = int(rng.integers(0, nodes))
        if x not in chal:
            chal.append(x)
    taken = set(chal)

    def parent_index():
        while True:
            x = int(rng.integers(0, nodes))
            if x not in taken:
                return x

    columns, graph = {}, []
    for c in chal:
        drg = [parent_index() for _ in range(6)]
        exp = [parent_index() for _ in range(8)]
        for p in drg + exp:
            if p not in columns:
                columns[p] = [rand() >> 2 for _ in range(L)]  # labels are 254-bit values
        graph.append((drg, exp))
    replica_id = rand()
    rid = replica_id.to_bytes(32, "little")
    # the challenged columns: layer 1 over the 6 DRG parents, layers 2.. over 6 DRG + 8 expander parents
    for c in chal:
        columns[c] = [None] * L
    for first in (True, False):
        lay, nod, par = [], [], bytearray()
        for c, (drg, exp) in zip(chal, graph):
            for layer in ([1] if first else range(2, L + 1)):
                ps = [columns[p][layer - 1] for p in drg]
                if not first:
                    ps += [columns[p][layer - 2] for p in exp]
                lay.append(layer)
                nod.append(c)
                par += b"".join(v.to_bytes(32, "little") for v in ps)
        if not lay:
            continue
        out = tree.to_ints(sdr.create_labels(ctx, rid, lay, nod, bytes(par), 6 if first else 14))
        for (layer, c), v in zip(zip(lay, nod), out):
            columns[c][layer - 1] = v
    data = {c: rand() for c in chal}
    col_idx = sorted(columns)
    col_hash = dict(zip(col_idx, pos_hash(L, [v for i in col_idx for v in columns[i]])))
    comm_d, d_path = _sparse_tree(data, [2] * circuit.info["depth_d"],
                                  lambda a, flat: [_sha_node(flat[i], flat[i + 1]) for i in range(0, len(flat), 2)],
                                  rand)
    comm_c, c_path = _sparse_tree(col_hash, circuit.arities, pos_hash, rand)
    enc = {c: (data[c] + columns[c][L - 1]) % FR_MODULUS for c in chal}
    comm_r_last, r_path = _sparse_tree(enc, circuit.arities, pos_hash, rand)
    comm_r = pos_hash(2, [comm_c, comm_r_last])[0]
    challenges = []
    for c, (drg, exp) in zip(chal, graph):
        challenges.append({
            "index": c, "data_leaf": data[c], "d_siblings": [s[0] for s in d_path(c)],
            "r_siblings": r_path(c), "c_column": columns[c], "c_siblings": c_path(c),
            "drg": [(p, columns[p], c_path(p)) for p in drg], "exp": [(p, columns[p], c_path(p)) for p in exp]})
    return {"replica_id": replica_id, "comm_d": comm_d, "comm_r": comm_r, "comm_r_last": comm_r_last,
            "comm_c": comm_c, "challenges": challenges}


def slots_of(circuit: StackedCircuit, inst: dict) -> bytes:
    """instance_slots over an instance dict (synthetic_instance's / the test oracle's format)"""
    return instance_slots(circuit, inst["replica_id"], inst["comm_d"], inst["comm_r"], inst["comm_r_last"],
                          inst["comm_c"], inst["challenges"])
