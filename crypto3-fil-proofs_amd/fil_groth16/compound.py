"""Mirror of the reference's compound-proof partition plumbing around the Groth16 prover.

  partition_count                 core/partitions.hpp:36-38 and compound_proof.hpp:85-87
  circuit_proofs                  compound_proof::circuit_proofs (compound_proof.hpp:127-137):
                                  one Groth16 proof per partition / vanilla proof
  MultiProof                      multi_proof{circuit_proofs, verifying_key} (core/proof/multi_proof.hpp:38-58)
                                  serialised as P x 192 bytes (api/seal.hpp:306-308, constants.hpp:93)
  get_partitions_for_window_post  libs/filecoin/src/api/post.cpp:37-46
  shard_partitions                one process per GPU: partition k goes to rank k % world
"""
from .core import PROOF_BYTES, prove


def partition_count(partitions: int) -> int:
    """core/partitions.hpp:36-38: -1 -> 1, 0 -> -1, p -> p."""
    return 1 if partitions == -1 else (-1 if partitions == 0 else partitions)


def get_partitions_for_window_post(total_sector_count: int, sector_count: int):
    """libs/filecoin/src/api/post.cpp:37-46.

    The reference computes ``std::ceil(total_sector_count / config.sector_count)`` on two size_t
    values, i.e. the ceil of an already-truncated integer quotient; that behaviour is kept.
    Returns None when the result is <= 1 (the reference's empty optional)."""
    partitions = total_sector_count // sector_count
    return partitions if partitions > 1 else None


class MultiProof:
    def __init__(self, proofs, verifying_key=None):
        self.circuit_proofs = list(proofs)
        self.verifying_key = verifying_key

    def size(self):
        return len(self.circuit_proofs)

    def empty(self):
        return not self.circuit_proofs

    def to_bytes(self) -> bytes:
        for p in self.circuit_proofs:
            assert len(p) == PROOF_BYTES
        return b"".join(self.circuit_proofs)

    @classmethod
    def from_bytes(cls, buf: bytes, verifying_key=None):
        if len(buf) % PROOF_BYTES:
            raise ValueError("multi-proof length is not a multiple of 192")
        return cls([buf[i:i + PROOF_BYTES] for i in range(0, len(buf), PROOF_BYTES)], verifying_key)


def circuit_proofs(ctx, pk, circuit, witnesses, blindings, priority=False):
    """One proof per partition, in partition order (compound_proof.hpp:127-137)."""
    if not witnesses:
        raise ValueError("Cannot create a circuit proof over missing vanilla proofs")
    if len(witnesses) != len(blindings):
        raise ValueError("one (r, s) pair per partition is required")
    return [prove(ctx, pk, circuit, z, r, s, priority=priority) for z, (r, s) in zip(witnesses, blindings)]


def shard_partitions(num_partitions: int, rank: int, world: int):
    """Partition indices proven by ``rank`` (round-robin: 10 partitions on 8 GPUs -> 2 rounds on 2)."""
    return list(range(rank, num_partitions, world))
