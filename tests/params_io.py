"""Test helper: bellman ``Parameters::write`` / ``VerifyingKey::write`` byte layout (the layout of
filecoin v28-*.params / *.vk files, mmapped by the reference's mapped_scheme_params,
core/crypto/mapped_scheme_params.hpp:43-84), written from the oracle's exported key."""
import struct


def vk_bytes(ex):
    return ex["vk"] + struct.pack(">I", len(ex["ic"]) // 96) + ex["ic"]


def params_bytes(ex):
    out = [vk_bytes(ex)]
    for key, esz in (("h", 96), ("l", 96), ("a", 96), ("b_g1", 96), ("b_g2", 192)):
        out.append(struct.pack(">I", len(ex[key]) // esz))
        out.append(ex[key])
    return b"".join(out)
