"""One process per GPU: shard independent partition proofs, gather the 192-byte proofs to rank 0.

Reference behaviour being distributed: compound_proof::circuit_proofs proves every partition of
a PoRep (10 at 32 GiB, proofs/constants.hpp:70-73) or Window-PoSt batch (post.cpp:37-46)
sequentially in-process and concatenates 192 x P bytes (api/seal.hpp:306-308).  Partitions are
independent proofs over the same proving key, so there is no data-path collective: each rank
proves partitions rank, rank + world, ... against its own resident key, and the only exchange is
one all-gather of the finished proofs (RCCL over xGMI with backend "nccl"; gloo on CPU tests).
"""
import numpy as np

from .compound import shard_partitions
from .core import PROOF_BYTES, SHARE_BYTES


def gather_multiproof(local_proofs, num_partitions: int, rank: int, world: int, device="cpu"):
    """local_proofs: this rank's proofs, in the order of shard_partitions(num_partitions, rank, world).
    Returns the P x 192-byte multi-proof (partition order) on every rank."""
    import torch
    import torch.distributed as dist

    mine = shard_partitions(num_partitions, rank, world)
    if len(local_proofs) != len(mine):
        raise ValueError(f"rank {rank} holds {len(local_proofs)} proofs, expected {len(mine)}")
    kmax = (num_partitions + world - 1) // world
    buf = np.zeros((kmax, PROOF_BYTES), dtype=np.uint8)
    for i, p in enumerate(local_proofs):
        if len(p) != PROOF_BYTES:
            raise ValueError("proofs are 192 bytes")
        buf[i] = np.frombuffer(p, dtype=np.uint8)
    t = torch.from_numpy(buf).to(device)
    if world > 1:
        bufs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(bufs, t)
        allp = [b.cpu().numpy() for b in bufs]
    else:
        allp = [t.cpu().numpy()]
    out = bytearray()
    for p in range(num_partitions):
        out += allp[p % world][p // world].tobytes()
    return bytes(out)


def prove_partitions(prove_fn, num_partitions: int, rank: int, world: int, device="cpu"):
    """Config-5 runner (Window-PoSt batch / PoRep C2 partitions over the GPUs of one node): this rank
    proves its round-robin share shard_partitions(P, rank, world) with ``prove_fn(partition_ids) ->
    list of 192-byte proofs`` (on a GPU: one fg.prove_batch over its witnesses, so partition k + 1's
    upload overlaps proof k), then the P x 192-byte multi-proof is all-gathered in partition order
    (api/seal.hpp:306-308; FallbackPoStCompound::prove per partition, api/post.hpp:305-348).
    10 partitions on 8 GPUs leave two rounds on ranks 0 and 1 (post.cpp:37-46, constants.hpp:88)."""
    mine = shard_partitions(num_partitions, rank, world)
    local = list(prove_fn(mine)) if mine else []
    return gather_multiproof(local, num_partitions, rank, world, device)


def gather_shares(share: bytes, world: int, device="cpu"):
    """All-gather one MI_SHARE_BYTES record per rank (the latency mode's only exchange, 576 B per GPU)."""
    import torch
    import torch.distributed as dist

    if len(share) != SHARE_BYTES:
        raise ValueError(f"shares are {SHARE_BYTES} bytes")
    t = torch.from_numpy(np.frombuffer(share, dtype=np.uint8).copy()).to(device)
    if world == 1:
        return [share]
    bufs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(bufs, t)
    return [b.cpu().numpy().tobytes() for b in bufs]


def prove_split(ctx, pk, circuit, z, r, s, rank: int, world: int, device="cpu", want_raw=False):
    """Single-proof latency mode: one proof over `world` ranks, one GPU each.

    Every rank holds the full proving key and witness, runs the witness map and NTT chain itself
    (no 2 GB H broadcast), and computes its contiguous slice of each MSM; the 576-byte shares are
    all-gathered and every rank assembles the same 192-byte proof as ``prove`` on one GPU."""
    from .core import assemble, prove_share

    vk, _ = pk.verifying_key()
    shares = gather_shares(prove_share(ctx, pk, circuit, z, rank, world), world, device)
    return assemble(vk, shares, r, s, want_raw=want_raw)
