"""Python mirror of the stacked-PoRep tree builders and the Poseidon hasher, over the C ABI
(include/mi355x_groth16.h, "Poseidon and the stacked-PoRep Merkle trees").

Reference names kept (paths relative to /root/reference/libs/storage/include/nil/filecoin/storage/proofs):
  * ``hash_single_column``   porep/stacked/vanilla/hash.hpp:37-47 (Poseidon over one column of labels)
  * ``ColumnTreeBuilder``    the builder generate_tree_c_gpu drives (porep/stacked/vanilla/proof.hpp:398-590):
                             ``add_final_columns`` -> (base_data, tree_data)
  * ``TreeBuilder``          the builder generate_tree_r_last drives (proof.hpp:630-760):
                             ``add_final_leaves`` -> tree_data
  * ``encode``               replica node = label + data node (proof.hpp:668-676)
  * ``get_merkle_tree_cache_size``  the cached-rows size the reference asserts (proof.hpp:717-721)
Values are canonical Fr: ints < r, or 32-byte little-endian strings.  Errors raise FilGpuError
(non-canonical inputs: MI_ERR_ARG), like the reference's asserts / throws.
"""
import ctypes

import numpy as np

from ._lib import check, lib, torch_sync
from .core import FR_MODULUS, _ptr

ARITIES = (2, 4, 8, 11)


def _fr_array(values) -> np.ndarray:
    """ints / 32-byte strings / uint8 array -> contiguous uint8 array of 32-byte LE entries."""
    if isinstance(values, np.ndarray):
        a = np.ascontiguousarray(values, dtype=np.uint8).reshape(-1)
        assert a.size % 32 == 0
        return a
    if isinstance(values, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(values), dtype=np.uint8).copy()
    out = bytearray()
    for v in values:
        out += v if isinstance(v, (bytes, bytearray)) else int(v).to_bytes(32, "little")
    return np.frombuffer(bytes(out), dtype=np.uint8).copy()


def to_ints(buf) -> list:
    b = bytes(buf)
    return [int.from_bytes(b[i:i + 32], "little") for i in range(0, len(b), 32)]


def poseidon_constants(arity: int):
    """(t, R_F, R_P, round_constants, mds) of the library's Poseidon for `arity` (canonical ints)."""
    shape = (ctypes.c_uint32 * 3)()
    check(lib().mi_poseidon_constants(arity, None, None, shape))
    t, rf, rp = shape
    rc = ctypes.create_string_buffer(32 * (rf + rp) * t)
    mds = ctypes.create_string_buffer(32 * t * t)
    check(lib().mi_poseidon_constants(arity, rc, mds, shape))
    m = to_ints(mds.raw)
    return t, rf, rp, to_ints(rc.raw), [m[i * t:(i + 1) * t] for i in range(t)]


def get_merkle_tree_cache_size(leafs: int, arity: int, rows_to_discard: int = 0) -> int:
    out = ctypes.c_uint64()
    check(lib().mi_tree_cache_size(leafs, arity, rows_to_discard, ctypes.byref(out)))
    return out.value


def default_rows_to_discard(leafs: int, arity: int) -> int:
    """merkletree's default: 2 rows above the base, never all rows but the root."""
    rows, n = 1, leafs
    while n > 1:
        n //= arity
        rows += 1
    return 0 if rows <= 2 else min(rows - 2, 2)


def poseidon_hash(ctx, arity: int, preimages) -> bytes:
    """digests (32 B each) of len(preimages) / arity hashes over consecutive groups of `arity` inputs."""
    a = _fr_array(preimages)
    n = a.size // 32 // arity
    assert n * arity * 32 == a.size, "preimages must be a multiple of arity"
    out = ctypes.create_string_buffer(32 * max(n, 1))
    p, keep = _ptr(a)
    check(lib().mi_poseidon_hash(ctx.h, arity, p, n, out))
    return out.raw[:32 * n]


def poseidon_hash_dev(ctx, arity: int, in_ptr: int, count: int, out_ptr: int):
    torch_sync(ctx)
    check(lib().mi_poseidon_hash_dev(ctx.h, arity, ctypes.c_void_p(in_ptr), count, ctypes.c_void_p(out_ptr)))


def hash_single_column(ctx, column) -> bytes:
    """porep/stacked/vanilla/hash.hpp:37-47: Poseidon over one column (2 or 11 labels)."""
    col = _fr_array(column)
    assert col.size // 32 in (2, 11), f"unsupported column size: {col.size // 32}"
    return poseidon_hash(ctx, col.size // 32, col)


class TreeBuilder:
    """TreeBuilder<Arity>: add_final_leaves(leaves) -> tree_data (every row above the base except the
    rows_to_discard lowest ones), bottom-up."""

    def __init__(self, ctx, arity: int = 8, rows_to_discard: int = 0):
        assert arity in ARITIES
        self.ctx, self.arity, self.rows_to_discard = ctx, arity, rows_to_discard

    def add_final_leaves(self, leaves) -> bytes:
        a = _fr_array(leaves)
        n = a.size // 32
        size = get_merkle_tree_cache_size(n, self.arity, self.rows_to_discard)
        out = ctypes.create_string_buffer(32 * max(size, 1))
        p, keep = _ptr(a)
        check(lib().mi_tree_build(self.ctx.h, self.arity, p, n, self.rows_to_discard, out))
        return out.raw[:32 * size]


class ColumnTreeBuilder:
    """ColumnTreeBuilder<ColumnArity, TreeArity>: add_final_columns(layers) -> (base_data, tree_data).
    `layers` is a list of ColumnArity per-layer label vectors (node j of column j = layers[l][j])."""

    def __init__(self, ctx, column_arity: int = 11, tree_arity: int = 8):
        assert column_arity in ARITIES and tree_arity in ARITIES
        self.ctx, self.column_arity, self.tree_arity = ctx, column_arity, tree_arity

    def add_final_columns(self, layers):
        assert len(layers) == self.column_arity
        arrs = [_fr_array(l) for l in layers]
        nodes = arrs[0].size // 32
        assert all(x.size == nodes * 32 for x in arrs)
        size = get_merkle_tree_cache_size(nodes, self.tree_arity, 0)
        ptrs = (ctypes.c_void_p * len(arrs))(*[x.ctypes.data for x in arrs])
        base = ctypes.create_string_buffer(32 * nodes)
        tree = ctypes.create_string_buffer(32 * max(size, 1))
        check(lib().mi_tree_c_build(self.ctx.h, self.column_arity, nodes, ptrs, self.tree_arity, base, tree))
        return base.raw, tree.raw[:32 * size]

    def add_final_columns_dev(self, labels_ptr: int, nodes: int, base_ptr: int, tree_ptr: int):
        """device variant: labels layer-major at labels_ptr (layer l at entry l * nodes)."""
        torch_sync(self.ctx)
        check(lib().mi_tree_c_build_dev(self.ctx.h, self.column_arity, nodes, ctypes.c_void_p(labels_ptr),
                                        self.tree_arity, ctypes.c_void_p(base_ptr), ctypes.c_void_p(tree_ptr)))


def generate_tree_r_last(ctx, last_layer_labels, data, arity: int = 8, rows_to_discard: int = 0):
    """encode every node (replica = label + data) and build the tree over the replica.
    Returns (replica bytes, tree_data bytes)."""
    lab = _fr_array(last_layer_labels)
    dat = _fr_array(data).copy()
    nodes = lab.size // 32
    assert dat.size == lab.size
    size = get_merkle_tree_cache_size(nodes, arity, rows_to_discard)
    tree = ctypes.create_string_buffer(32 * max(size, 1))
    pl, k1 = _ptr(lab)
    pd, k2 = _ptr(dat)
    check(lib().mi_tree_r_last_build(ctx.h, nodes, pl, pd, arity, rows_to_discard, tree))
    return dat.tobytes(), tree.raw[:32 * size]


def generate_tree_r_last_dev(ctx, nodes: int, labels_ptr: int, data_ptr: int, tree_ptr: int, arity: int = 8,
                             rows_to_discard: int = 0):
    torch_sync(ctx)
    check(lib().mi_tree_r_last_build_dev(ctx.h, nodes, ctypes.c_void_p(labels_ptr), ctypes.c_void_p(data_ptr),
                                         arity, rows_to_discard, ctypes.c_void_p(tree_ptr)))


def encode(key: int, value: int) -> int:
    return (key + value) % FR_MODULUS


def tree_height(leafs: int, arity: int) -> int:
    h = 0
    while leafs > 1:
        leafs //= arity
        h += 1
    return h


def gen_proofs_dev(ctx, arity: int, leaves_ptr: int, leafs: int, rows_to_discard: int, tree_ptr: int, count: int,
                   challenges_ptr: int, leaf_out_ptr: int, siblings_out_ptr: int) -> None:
    """Inclusion proofs of `count` challenges (u64 leaf indices) in a device-resident tree (MerkleTree_gen_proof /
    MerkleTree_gen_cached_proof, porep/stacked/vanilla/proof.hpp:139-140,183-186): the leaf, then per row
    j = 0 .. height-1 the arity - 1 siblings in position order skipping the path's own slot (digit j of the
    challenge in base arity).  tree_ptr holds the cached rows built with the same rows_to_discard."""
    vp = ctypes.c_void_p
    torch_sync(ctx)
    check(lib().mi_tree_inclusion_paths_dev(ctx.h, arity, vp(leaves_ptr), leafs, rows_to_discard, vp(tree_ptr), count,
                                            vp(challenges_ptr), vp(leaf_out_ptr), vp(siblings_out_ptr)))

