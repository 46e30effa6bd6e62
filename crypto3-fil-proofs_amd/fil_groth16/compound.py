"""Mirror of the reference's compound-proof partition plumbing around the Groth16 prover.

  partition_count                 core/partitions.hpp:36-38 and compound_proof.hpp:85-87
  circuit_proofs                  compound_proof::circuit_proofs (compound_proof.hpp:127-137):
                                  one Groth16 proof per partition / vanilla proof
  MultiProof                      multi_proof{circuit_proofs, verifying_key} (core/proof/multi_proof.hpp:38-58)
                                  serialised as P x 192 bytes (api/seal.hpp:306-308, constants.hpp:93)
  MultiProof.verify               verify_seal's Groth16 batch check of all partitions (api/seal.hpp:339-485)
  seal_commit_phase2_proofs       the C2 tail (api/seal.hpp:296-313): circuit_proofs -> MultiProof ->
                                  self-verification ("post-seal verification sanity check failed")
  get_partitions_for_window_post  libs/filecoin/src/api/post.cpp:37-46
  generate_window_post_proofs     generate_window_post (api/post.hpp:305-348): partitions from the sector
                                  count, FallbackPoStCompound::prove over them with post_config.priority
  generate_winning_post_proof     generate_winning_post (api/post.hpp:178-230): one partition
  shard_partitions                one process per GPU: partition k goes to rank k % world
  select_challenges               proofs/parameters.hpp:90-99 (LayerChallenges, porep/stacked/vanilla/challenges.hpp:44-48)
  porep_layer_challenges          setup_params' challenge selection for a sector size (parameters.hpp:78-88,
                                  POREP_MINIMUM_CHALLENGES / POREP_PARTITIONS / LAYERS, constants.hpp:65-78)
"""
from collections import namedtuple

from .core import PROOF_BYTES, prove, prove_batch, verify_batch


def partition_count(partitions: int) -> int:
    """core/partitions.hpp:36-38: -1 -> 1, 0 -> -1, p -> p."""
    return 1 if partitions == -1 else (-1 if partitions == 0 else partitions)


# porep/stacked/vanilla/challenges.hpp:44-48: {layers, max_count}; challenges_count_all() is max_count (the
# reference's test pins it: select_challenges(p, 12, 11).challenges_count_all() = 12 / 6 / 3 for p = 1 / 2 / 4,
# libs/filecoin/test/parameters.cpp:35-43)
LayerChallenges = namedtuple("LayerChallenges", ["layers", "max_count"])
LayerChallenges.challenges_count_all = lambda self: self.max_count

SECTOR_SIZE_32GIB = 1 << 35
SECTOR_SIZE_64GIB = 1 << 36
# constants.hpp:65-78 (every smaller sector size: 2 challenges, 1 partition, 2 layers)
POREP_MINIMUM_CHALLENGES = {SECTOR_SIZE_32GIB: 176, SECTOR_SIZE_64GIB: 176}
POREP_PARTITIONS = {SECTOR_SIZE_32GIB: 10, SECTOR_SIZE_64GIB: 10}
LAYERS = {SECTOR_SIZE_32GIB: 11, SECTOR_SIZE_64GIB: 11}


def select_challenges(partitions: int, minimum_total_challenges: int, layers: int) -> LayerChallenges:
    """proofs/parameters.hpp:90-99: the smallest per-partition challenge count whose total over the partitions
    reaches the minimum."""
    if partitions < 1:
        raise ValueError("select_challenges: partitions must be >= 1")
    count = 1
    guess = LayerChallenges(layers, count)
    while partitions * guess.challenges_count_all() < minimum_total_challenges:
        count += 1
        guess = LayerChallenges(layers, count)
    return guess


def porep_layer_challenges(sector_bytes: int) -> LayerChallenges:
    """The LayerChallenges setup_params derives for a sector size (parameters.hpp:78-88): 32 / 64 GiB -> 11 layers x
    18 challenges per partition (176 over 10 partitions); the small test sizes -> 2 layers x 2 challenges."""
    return select_challenges(POREP_PARTITIONS.get(sector_bytes, 1), POREP_MINIMUM_CHALLENGES.get(sector_bytes, 2),
                             LAYERS.get(sector_bytes, 2))


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

    def verify(self, public_inputs, seed=None) -> bool:
        """Batch-verify every partition proof against ``verifying_key`` = (vk, ic) with the per-partition
        public inputs (without ONE).  One multi-pairing, random weights from ``seed``."""
        if self.verifying_key is None:
            raise ValueError("multi-proof has no verifying key")
        vk, ic = self.verifying_key
        if len(public_inputs) != len(self.circuit_proofs):
            raise ValueError("one public-input vector per partition is required")
        return verify_batch(vk, ic, list(public_inputs), self.circuit_proofs, seed)

    @classmethod
    def from_bytes(cls, buf: bytes, verifying_key=None):
        if len(buf) % PROOF_BYTES:
            raise ValueError("multi-proof length is not a multiple of 192")
        return cls([buf[i:i + PROOF_BYTES] for i in range(0, len(buf), PROOF_BYTES)], verifying_key)


def circuit_proofs(ctx, pk, circuit, witnesses, blindings=None, priority=False):
    """One proof per partition, in partition order (compound_proof.hpp:127-137), through the batch entry
    the bench times (mi_groth16_prove_batch: partition k + 1's witness upload and proof k's host assembly
    overlap proof k's GPU work).  blindings = None is the production call: r, s drawn inside the library
    (crypto3 prove's internal randomness); explicit (r, s) pairs are the parity/test entry."""
    if not witnesses:
        raise ValueError("Cannot create a circuit proof over missing vanilla proofs")
    if blindings is not None and len(witnesses) != len(blindings):
        raise ValueError("one (r, s) pair per partition is required")
    ws = list(witnesses)
    on_device = [isinstance(z, int) for z in ws]
    if any(on_device):  # witnesses already in HBM (e.g. the library-built circuits' GPU witness): one prove each
        if not all(on_device):
            raise TypeError("witnesses must be all host buffers or all device pointers")
        return [prove(ctx, pk, circuit, z, *(blindings[k] if blindings is not None else (None, None)),
                      priority=priority) for k, z in enumerate(ws)]
    return prove_batch(ctx, pk, circuit, ws, blindings, priority=priority)


def seal_commit_phase2_proofs(ctx, pk, circuit, witnesses, blindings=None, num_inputs=None,
                              priority=False, public_inputs=None) -> bytes:
    """api/seal.hpp:296-313: prove every partition, pack the MultiProof buffer and refuse to return
    one that does not verify.  ``witnesses`` are full assignments (ONE first), in host memory or as device
    pointers; the public inputs of partition k are its witness entries 1 .. num_inputs - 1 (device
    witnesses: given as ``public_inputs``, e.g. StackedCircuit.public_inputs of each partition's slots)."""
    if num_inputs is None:
        num_inputs = circuit.num_inputs
    proofs = circuit_proofs(ctx, pk, circuit, witnesses, blindings, priority=priority)
    mp = MultiProof(proofs, pk.verifying_key())
    if public_inputs is None:
        if any(isinstance(z, int) for z in witnesses):
            raise ValueError("device witnesses: pass public_inputs (one 32 x (num_inputs - 1)-byte vector each)")
        public_inputs = [bytes(z[32:32 * num_inputs]) for z in witnesses]
    inputs = list(public_inputs)
    if not mp.verify(inputs):
        raise RuntimeError("post-seal verification sanity check failed")
    return mp.to_bytes()


def shard_partitions(num_partitions: int, rank: int, world: int):
    """Partition indices proven by ``rank`` (round-robin: 10 partitions on 8 GPUs -> 2 rounds on 2)."""
    return list(range(rank, num_partitions, world))


def _post_partitions(num_sectors: int, sector_count: int) -> int:
    """The partition count FallbackPoStCompound::setup receives: get_partitions_for_window_post's
    optional, unset (None) meaning one partition (compound_proof.hpp:85-87 partition_count(-1) = 1)."""
    p = get_partitions_for_window_post(num_sectors, sector_count)
    return partition_count(-1 if p is None else p)


def generate_window_post_proofs(ctx, pk, circuit, num_sectors: int, sector_count: int, witnesses, blindings=None,
                                priority: bool = True) -> bytes:
    """api/post.hpp:305-348: the Window-PoSt SNARK.  ``witnesses`` holds one synthesised assignment per
    partition (circuit synthesis is upstream of the boundary); their number must equal the partition
    count derived from (num_sectors, sector_count) exactly as the reference derives it.  Proofs are made
    on the high-priority stream when ``priority`` (post_config.priority, types/post_config.hpp:41-42) and
    returned as the P x 192-byte proof vector (proof.to_vec())."""
    parts = _post_partitions(num_sectors, sector_count)
    if len(witnesses) != parts:
        raise ValueError(f"window post: {parts} partition(s) for {num_sectors} sectors of {sector_count}, "
                         f"got {len(witnesses)} witness(es)")
    return MultiProof(circuit_proofs(ctx, pk, circuit, witnesses, blindings, priority=priority)).to_bytes()


def generate_winning_post_proof(ctx, pk, circuit, num_replicas: int, sector_count: int, witness, blinding=None,
                                priority: bool = False) -> bytes:
    """api/post.hpp:178-230: the Winning-PoSt SNARK -- exactly ``sector_count`` replicas ("invalid amount
    of replicas"), partitions unset (one partition), one 192-byte proof."""
    if num_replicas != sector_count:
        raise ValueError("invalid amount of replicas")
    return MultiProof(circuit_proofs(ctx, pk, circuit, [witness], None if blinding is None else [blinding],
                                     priority=priority)).to_bytes()
