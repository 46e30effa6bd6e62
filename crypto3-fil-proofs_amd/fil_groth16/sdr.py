"""Python mirror of the stacked-PoRep labelling witness over the C ABI (include/mi355x_groth16.h,
"SDR labelling witness").

Reference names kept (paths relative to /root/reference/libs/storage/include/nil/filecoin/storage/proofs):
  * ``LabelingProof``       porep/stacked/vanilla/labelling_proof.hpp:40-48 (parents, layer_index, node) with
                            ``create_label`` / ``verify`` as in vanilla/detail/processing/naive/labelling_proof.hpp:46-70
  * ``EncodingProof``       porep/stacked/vanilla/encoding_proof.hpp:37-70: ``create_key`` (the same hash) and
                            ``verify`` (encode(key, decoded) == encoded, encode = addition in Fr)
  * ``create_labels``       many LabelingProof::create_label calls in one launch
  * ``labeling_proofs_dev`` the per-challenge loop of prove_layers (vanilla/proof.hpp:190-255): parents gathered
                            from the device-resident layer labels, base parents from the challenged layer and
                            expander parents from the layer below, repeated to TOTAL_PARENTS = 37
The label is SHA-256(replica_id || u32_be(layer) || u64_be(node) || 0^20 || 37 parents) with the top two bits
of byte 31 cleared (create_label.hpp:76-77), a canonical Fr in little-endian bytes.
"""
import ctypes
from dataclasses import dataclass
from typing import List

import numpy as np

from ._lib import check, lib, torch_sync
from .core import FR_MODULUS, _ptr

TOTAL_PARENTS = 37  # vanilla/proof.hpp:49
BASE_DEGREE = 6     # core/drgraph.hpp (DRG parents, current layer)
EXP_DEGREE = 8      # vanilla/graph.hpp:37 (expander parents, previous layer)
NODE_SIZE = 32


def repeat_parents(parents: List[bytes]) -> List[bytes]:
    """parents_data_full: the parents repeated cyclically to TOTAL_PARENTS (vanilla/proof.hpp:233-237)."""
    if not parents:
        return []
    return [parents[k % len(parents)] for k in range(TOTAL_PARENTS)]


def create_labels(ctx, replica_id: bytes, layers, nodes, parents, n_parents: int) -> bytes:
    """Labels of many (layer, node) pairs in one launch.  parents: n_parents 32-byte labels per entry
    (bytes / uint8 array, entry-major), repeated to 37 on the device; n_parents = 0 gives node 0's label."""
    lay = np.ascontiguousarray(layers, dtype=np.uint32)
    nod = np.ascontiguousarray(nodes, dtype=np.uint64)
    n = lay.size
    if nod.size != n or len(replica_id) != 32:
        raise ValueError("layers and nodes must have the same length; replica_id is 32 bytes")
    par = np.frombuffer(bytes(parents), dtype=np.uint8) if n_parents else np.zeros(1, np.uint8)
    if n_parents and par.size != 32 * n_parents * n:
        raise ValueError("parents must hold n_parents 32-byte labels per entry")
    out = np.empty(32 * max(n, 1), dtype=np.uint8)
    rp, k1 = _ptr(bytes(replica_id))
    pp, k2 = _ptr(par)
    check(lib().mi_sdr_labels(ctx.h, rp, n, ctypes.c_void_p(lay.ctypes.data), ctypes.c_void_p(nod.ctypes.data),
                              pp, n_parents, ctypes.c_void_p(out.ctypes.data)))
    return out[:32 * n].tobytes()


def create_labels_dev(ctx, replica_id: bytes, count: int, layers_dev: int, nodes_dev: int, parents_dev: int,
                      n_parents: int, labels_dev: int) -> None:
    """Device-resident form of create_labels (raw device pointers, e.g. torch tensor data_ptr())."""
    rp, k = _ptr(bytes(replica_id))
    torch_sync(ctx)
    check(lib().mi_sdr_labels_dev(ctx.h, rp, count, ctypes.c_void_p(layers_dev), ctypes.c_void_p(nodes_dev),
                                  ctypes.c_void_p(parents_dev), n_parents, ctypes.c_void_p(labels_dev)))


def labeling_proofs_dev(ctx, replica_id: bytes, n_layers: int, nodes_per_layer: int, layer_labels_dev: int,
                        count: int, layers_dev: int, challenges_dev: int, parent_idx_dev: int,
                        labels_dev: int, parents_out_dev: int = 0, n_base: int = BASE_DEGREE,
                        n_exp: int = EXP_DEGREE) -> None:
    """Labels (and optionally parents_data_full) of `count` challenges, parents gathered on the device from
    the layer-major labels by parent_idx (u32, n_base + n_exp per challenge).  Out-of-range layers or parent
    indices raise FilGpuError (MI_ERR_ARG) before any gather."""
    rp, k = _ptr(bytes(replica_id))
    vp = ctypes.c_void_p
    torch_sync(ctx)
    check(lib().mi_sdr_labeling_proofs_dev(ctx.h, rp, n_layers, nodes_per_layer, vp(layer_labels_dev), count,
                                           vp(layers_dev), vp(challenges_dev), vp(parent_idx_dev), n_base, n_exp,
                                           vp(labels_dev), vp(parents_out_dev or None)))


@dataclass
class LabelingProof:
    """vanilla/labelling_proof.hpp:40-48: the 37 parent labels of a challenged node at one layer."""
    parents: List[bytes]
    layer_index: int
    node: int

    def create_label(self, ctx, replica_id: bytes) -> bytes:
        return create_labels(ctx, replica_id, [self.layer_index], [self.node], b"".join(self.parents),
                             len(self.parents))

    def verify(self, ctx, replica_id: bytes, expected_label: bytes) -> bool:
        return self.create_label(ctx, replica_id) == bytes(expected_label)


def encode(key: bytes, value: bytes) -> bytes:
    """encode(key, value) = key + value in Fr (32-byte LE; the replica node, proof.hpp:668-676)."""
    k, v = int.from_bytes(key, "little"), int.from_bytes(value, "little")
    if k >= FR_MODULUS or v >= FR_MODULUS:
        raise ValueError("encode: operands must be canonical Fr")
    return ((k + v) % FR_MODULUS).to_bytes(32, "little")


@dataclass
class EncodingProof:
    """vanilla/encoding_proof.hpp:37-70."""
    parents: List[bytes]
    layer_index: int
    node: int

    def create_key(self, ctx, replica_id: bytes) -> bytes:
        return LabelingProof(self.parents, self.layer_index, self.node).create_label(ctx, replica_id)

    def verify(self, ctx, replica_id: bytes, exp_encoded_node: bytes, decoded_node: bytes) -> bool:
        return encode(self.create_key(ctx, replica_id), decoded_node) == bytes(exp_encoded_node)


def build_tree_d_dev(ctx, leaves_ptr: int, leafs: int, tree_ptr: int) -> None:
    """tree D over 32-byte data nodes on the device (node = SHA256(left || right), byte 31 &= 0x3f): every row
    above the leaves, bottom-up, leafs - 1 entries.  Openings: tree_d_proofs_dev."""
    torch_sync(ctx)
    check(lib().mi_tree_d_build_dev(ctx.h, ctypes.c_void_p(leaves_ptr), leafs, ctypes.c_void_p(tree_ptr)))


def tree_d_proofs_dev(ctx, leaves_ptr: int, leafs: int, tree_ptr: int, count: int, challenges_ptr: int,
                      leaf_out_ptr: int, siblings_out_ptr: int) -> None:
    """Inclusion proofs in a device-resident tree D (MerkleTree_gen_proof(tree_d), vanilla/proof.hpp:139-140):
    the layouts of tree.gen_proofs_dev at arity 2; every row is cached, so nothing is rebuilt (a rebuild would
    need SHA-256, and tree.gen_proofs_dev rebuilds discarded rows with Poseidon)."""
    vp = ctypes.c_void_p
    torch_sync(ctx)
    check(lib().mi_tree_d_inclusion_paths_dev(ctx.h, vp(leaves_ptr), leafs, vp(tree_ptr), count, vp(challenges_ptr),
                                              vp(leaf_out_ptr), vp(siblings_out_ptr)))
