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


SRS_PARTS = ("vk", "ic", "h", "l", "a", "b_g1", "b_g2")


def broadcast_srs_parts(parts, rank: int, world: int, src: int = 0, device="cpu", chunk_bytes: int = 1 << 30):
    """Broadcast a proving key in the bellman wire layout (dict of SRS_PARTS -> bytes, held by ``src``) to
    every rank: one size vector, then each part in chunks of at most ``chunk_bytes`` (large transfers over
    xGMI with backend "nccl" on device tensors, bounded staging memory).  The reference loads the same
    params file in every process (get_groth_params, core/parameter_cache.hpp:185-200); here one rank reads
    the file and the others receive it.  Returns the dict on every rank."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return dict(parts)
    sizes = torch.zeros(len(SRS_PARTS), dtype=torch.int64)
    if rank == src:
        sizes = torch.tensor([len(parts[k]) for k in SRS_PARTS], dtype=torch.int64)
    sizes = sizes.to(device)
    dist.broadcast(sizes, src)
    out = {}
    for k, n in zip(SRS_PARTS, sizes.cpu().tolist()):
        host = np.empty(n, dtype=np.uint8)
        src_view = np.frombuffer(parts[k], dtype=np.uint8) if rank == src else None
        for off in range(0, n, chunk_bytes):
            m = min(chunk_bytes, n - off)
            t = (torch.from_numpy(src_view[off:off + m].copy()) if rank == src
                 else torch.empty(m, dtype=torch.uint8)).to(device)
            dist.broadcast(t, src)
            host[off:off + m] = t.cpu().numpy()
        out[k] = host.tobytes()
    return out


def broadcast_proving_key(ctx, pk, circuit, rank: int, world: int, src: int = 0, device="cpu", checked=False,
                          chunk_bytes: int = 1 << 30):
    """Rank ``src`` holds ``pk`` (e.g. ProvingKey.load_params from a v28 file); every other rank receives
    the key over the process group and uploads it to its own GPU.  Returns this rank's ProvingKey."""
    from .core import ProvingKey

    parts = None
    if rank == src:
        vk, ic = pk.verifying_key()
        parts = dict(vk=vk, ic=ic, h=pk.query(0), l=pk.query(1), a=pk.query(2), b_g1=pk.query(3),
                     b_g2=pk.query(4))
    parts = broadcast_srs_parts(parts, rank, world, src, device, chunk_bytes)
    if rank == src:
        return pk
    return ProvingKey.load(ctx, circuit, *(parts[k] for k in SRS_PARTS), checked=checked)
