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


def _group_active(world: int) -> bool:
    """True when a process group is initialised (then every exchange goes through it, a world of one
    included: that is how a one-GPU box runs the RCCL path); it must have ``world`` ranks."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        if world > 1:
            raise RuntimeError(f"world size {world} needs an initialised process group")
        return False
    if dist.get_world_size() != world:
        raise ValueError(f"process group has {dist.get_world_size()} ranks, caller says {world}")
    return True


def _all_gather(t, world: int):
    """all_gather of one tensor per rank over the process group (RCCL for device tensors with "nccl"),
    returned as host numpy arrays in rank order; a plain copy without a group."""
    import torch
    import torch.distributed as dist

    if not _group_active(world):
        return [t.cpu().numpy()]
    bufs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(bufs, t)
    return [b.cpu().numpy() for b in bufs]


def gather_multiproof(local_proofs, num_partitions: int, rank: int, world: int, device="cpu"):
    """local_proofs: this rank's proofs, in the order of shard_partitions(num_partitions, rank, world).
    Returns the P x 192-byte multi-proof (partition order) on every rank."""
    import torch

    mine = shard_partitions(num_partitions, rank, world)
    if len(local_proofs) != len(mine):
        raise ValueError(f"rank {rank} holds {len(local_proofs)} proofs, expected {len(mine)}")
    kmax = (num_partitions + world - 1) // world
    buf = np.zeros((kmax, PROOF_BYTES), dtype=np.uint8)
    for i, p in enumerate(local_proofs):
        if len(p) != PROOF_BYTES:
            raise ValueError("proofs are 192 bytes")
        buf[i] = np.frombuffer(p, dtype=np.uint8)
    allp = _all_gather(torch.from_numpy(buf).to(device), world)
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


def balanced_schedule(num_partitions: int, world: int):
    """Config-5 schedule without an idle tail.  Round-robin leaves P % W partitions for a last round in which
    W - P % W GPUs idle (10 partitions on 8 GPUs: two full rounds on ranks 0 and 1, six GPUs waiting).  Here
    the first P - P % W partitions go round-robin as whole proofs, and each of the R = P % W remaining ones
    is proven by a GROUP of ranks in latency mode (mi_groth16_prove_share: every rank of a group its slice
    of the five MSMs, the shares assembled on the host).  Groups partition the ranks: sizes W // R, the
    first W % R of them one larger.  A group of one rank proves its partition whole.
    -> (whole, tail): whole[r] = partitions rank r proves whole; tail = [(partition, [ranks])]."""
    if num_partitions < 0 or world < 1:
        raise ValueError("need num_partitions >= 0 and world >= 1")
    R = num_partitions % world
    full = num_partitions - R
    whole = [list(range(r, full, world)) for r in range(world)]
    tail, start = [], 0
    for j in range(R):
        g = world // R + (1 if j < world % R else 0)
        tail.append((full + j, list(range(start, start + g))))
        start += g
    for p, ranks in tail:
        if len(ranks) == 1:  # a group of one: a whole proof
            whole[ranks[0]].append(p)
    tail = [(p, ranks) for p, ranks in tail if len(ranks) > 1]
    return whole, tail


def agree_blinding(count: int, rank: int, device="cpu"):
    """``count`` (r, s) pairs drawn by rank 0 from the OS CSPRNG and broadcast, so that every rank of a group
    assembles the same proof from the gathered shares (bellman create_random_proof draws r, s once per
    proof; here the proof is assembled on several ranks)."""
    import os

    import torch
    import torch.distributed as dist

    from .core import FR_MODULUS

    t = torch.from_numpy(np.frombuffer(os.urandom(128 * count), dtype=np.uint8).copy()) if rank == 0 else \
        torch.zeros(128 * count, dtype=torch.uint8)
    t = t.to(device)
    dist.broadcast(t, 0)
    raw = t.cpu().numpy().tobytes()
    ints = [int.from_bytes(raw[64 * i:64 * (i + 1)], "little") % FR_MODULUS for i in range(2 * count)]
    return [(ints[2 * i], ints[2 * i + 1]) for i in range(count)]


MAX_SHARES = 2  # shares one rank contributes to a tail proof (H-split groups: its L/A/B slice, then its H slice)


_GROUPS = {}  # (ranks, device) -> process subgroup, created once per schedule (group_broadcaster)


def group_broadcaster(ranks, device="cpu"):
    """bcast(tensor) over the process subgroup ``ranks`` from its first rank (the group's lead), in place; every
    process must create the subgroups of a schedule in the same order (torch.distributed.new_group).  Without a
    process group (one rank) it is the identity.  The subgroup is created at the first call for these ranks and
    reused after it (every step of a schedule asks for the same groups, and each new RCCL communicator holds
    memory, streams and a lazy setup on its first broadcast); destroy_group_broadcasters frees them.  The first
    call also runs one small broadcast, so that setup lands outside the caller's timed steps."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return lambda t: (lambda: t)
    key = (tuple(ranks), str(device))
    pg = _GROUPS.get(key)
    if pg is None:
        pg = dist.new_group(list(ranks))  # collective over the whole world: same order on every rank
        if dist.get_rank() in ranks:
            dist.broadcast(torch.zeros(1, dtype=torch.uint8, device=device), ranks[0], group=pg)  # warm-up
        _GROUPS[key] = pg

    def bcast(t):
        """starts the broadcast of t (asynchronous: RCCL on its own stream); returns done() -> t, which waits for
        it (and orders torch's current stream after it, so the library's caller-stream fence covers the data)"""
        work = dist.broadcast(t, ranks[0], group=pg, async_op=True)

        def done():
            work.wait()
            return t

        return done

    return bcast


def destroy_group_broadcasters():
    """Frees the subgroups group_broadcaster created (collective: every rank calls it, in the same order)."""
    import torch.distributed as dist

    for key in list(_GROUPS):
        pg = _GROUPS.pop(key)
        if dist.is_available() and dist.is_initialized():
            dist.destroy_process_group(pg)


def prove_partitions_balanced(prove_fn, share_fn, assemble_fn, num_partitions: int, rank: int, world: int,
                              device="cpu", group_bcast=False):
    """prove_partitions with the balanced_schedule: ``prove_fn(ids) -> [192-byte proofs]`` for this rank's
    whole partitions, ``share_fn(partition, k, g) -> 576-byte share`` (or a list of up to MAX_SHARES of them)
    for its slice k of g of a tail partition, ``assemble_fn(partition, shares) -> 192-byte proof`` (fg.assemble
    with that partition's blinding, identical on every rank).  group_bcast: share_fn gets a fourth argument, the
    tail group's broadcaster (group_broadcaster: H coefficients from the lead, hsplit_shares).  One all-gather
    carries every rank's whole proofs and its shares; each rank then assembles the tail proofs itself.  Returns
    the P x 192-byte multi-proof (partition order) on every rank, byte-identical to prove_partitions' for the
    same blinding."""
    import torch

    whole, tail = balanced_schedule(num_partitions, world)
    bcasts = {p: group_broadcaster(ranks, device) for p, ranks in tail} if group_bcast else {}
    kmax = max((len(w) for w in whole), default=0)
    local = list(prove_fn(whole[rank])) if whole[rank] else []
    if len(local) != len(whole[rank]) or any(len(p) != PROOF_BYTES for p in local):
        raise ValueError(f"rank {rank}: prove_fn returned {len(local)} proofs for {len(whole[rank])} partitions")
    base = kmax * PROOF_BYTES
    rec = np.zeros(base + 1 + MAX_SHARES * SHARE_BYTES, dtype=np.uint8)
    for i, p in enumerate(local):
        rec[i * PROOF_BYTES:(i + 1) * PROOF_BYTES] = np.frombuffer(p, dtype=np.uint8)
    for p, ranks in tail:
        if rank in ranks:
            args = (p, ranks.index(rank), len(ranks)) + ((bcasts[p],) if group_bcast else ())
            got = share_fn(*args)
            shares = [got] if isinstance(got, (bytes, bytearray)) else list(got)
            if not 1 <= len(shares) <= MAX_SHARES or any(len(sh) != SHARE_BYTES for sh in shares):
                raise ValueError(f"one to {MAX_SHARES} shares of {SHARE_BYTES} bytes per rank")
            rec[base] = len(shares)
            for j, sh in enumerate(shares):
                rec[base + 1 + j * SHARE_BYTES:base + 1 + (j + 1) * SHARE_BYTES] = np.frombuffer(sh, dtype=np.uint8)
    allr = _all_gather(torch.from_numpy(rec).to(device), world)
    out = {}
    for r in range(world):
        for i, p in enumerate(whole[r]):
            out[p] = allr[r][i * PROOF_BYTES:(i + 1) * PROOF_BYTES].tobytes()
    for p, ranks in tail:
        sh = [allr[r][base + 1 + j * SHARE_BYTES:base + 1 + (j + 1) * SHARE_BYTES].tobytes()
              for r in ranks for j in range(int(allr[r][base]))]
        out[p] = assemble_fn(p, sh)
    return b"".join(out[p] for p in range(num_partitions))


def latency_ranges(sizes, group: int, lead_share: float = 0.0):
    """Query ranges of a latency-mode group of ``group`` ranks that computes H once (every rank of a
    group used to repeat the witness map and the NTT chain, ~317 ms per share of a 32 GiB Window-PoSt
    partition).  sizes = (n_h, n_l, n_a, n_b) of the proving key (ProvingKey.n_h ...).  Rank 0 of the group
    takes the whole H query -- it alone runs the witness map and the NTT chain -- plus the fraction
    ``lead_share`` of L, A and B; ranks 1 .. g - 1 split the rest of L, A and B into equal contiguous slices.
    Returns one [(first, count)] x 4 (H, L, A, B) list per rank; together they partition every query, so the
    assembled proof equals the one-GPU proof (mi_groth16_prove_share_ranges)."""
    if group < 1:
        raise ValueError("a group has at least one rank")
    if not 0.0 <= lead_share <= 1.0:
        raise ValueError("lead_share is a fraction")
    n_h, n_l, n_a, n_b = (int(x) for x in sizes)
    if group == 1:
        return [[(0, n_h), (0, n_l), (0, n_a), (0, n_b)]]
    out = [[(0, n_h)] + [None] * 3] + [[(n_h, 0)] + [None] * 3 for _ in range(group - 1)]
    for q, n in ((1, n_l), (2, n_a), (3, n_b)):
        n0 = int(round(n * lead_share))
        out[0][q] = (0, n0)
        rest = n - n0
        for k in range(1, group):
            lo = n0 + rest * (k - 1) // (group - 1)
            hi = n0 + rest * k // (group - 1)
            out[k][q] = (lo, hi - lo)
    return out


def latency_ranges_hsplit(sizes, group: int, h_lead: float, lab_lead: float = 0.0):
    """Query ranges of a latency group that computes H ONCE and SPLITS it: the lead (rank 0 of the
    group) runs the witness map and the NTT chain (mi_groth16_h_coeffs_dev), broadcasts the d H coefficients over
    the group, and takes the fraction ``h_lead`` of the H query plus ``lab_lead`` of L, A and B; ranks 1 .. g - 1
    split the rest of every query into equal contiguous slices.  One [(first, count)] x 4 (H, L, A, B) list per
    rank; together they partition every query (the assembled proof equals the one-GPU proof)."""
    if group < 1:
        raise ValueError("a group has at least one rank")
    if not (0.0 <= h_lead <= 1.0 and 0.0 <= lab_lead <= 1.0):
        raise ValueError("lead fractions are in [0, 1]")
    n = [int(x) for x in sizes]
    if group == 1:
        return [[(0, n[0]), (0, n[1]), (0, n[2]), (0, n[3])]]
    out = [[None] * 4 for _ in range(group)]
    for q in range(4):
        n0 = int(round(n[q] * (h_lead if q == 0 else lab_lead)))
        out[0][q] = (0, n0)
        rest = n[q] - n0
        for k in range(1, group):
            lo = n0 + rest * (k - 1) // (group - 1)
            hi = n0 + rest * k // (group - 1)
            out[k][q] = (lo, hi - lo)
    return out


def hsplit_fractions(t_qap: float, t_hmsm: float, t_lab: float, group: int):
    """(h_lead, lab_lead) that even out an H-split group: t_qap = witness map + NTT chain (the lead alone), t_hmsm =
    the whole H MSM, t_lab = L, A and B, all on one GPU.  The lead runs t_qap + h t_hmsm + f t_lab, every other rank
    ((1 - h) t_hmsm + (1 - f) t_lab) / (g - 1).  With f = 0: h = (t_lab + t_hmsm - (g - 1) t_qap) / (g t_hmsm); if
    that exceeds 1 the lead takes all of H and f = (t_lab - (g - 1)(t_qap + t_hmsm)) / (g t_lab); if it is negative
    the NTT chain alone outweighs a share (h = f = 0).  Clamped to [0, 1]."""
    if group <= 1:
        return 1.0, 1.0
    h = (t_lab + t_hmsm - (group - 1) * t_qap) / (group * t_hmsm) if t_hmsm > 0 else 1.0
    if h <= 1.0:
        return max(0.0, h), 0.0
    f = (t_lab - (group - 1) * (t_qap + t_hmsm)) / (group * t_lab) if t_lab > 0 else 0.0
    return 1.0, min(1.0, max(0.0, f))


def hsplit_shares(k: int, ranges, h_coeffs_fn, share_fn, bcast):
    """This rank's shares of an H-split tail proof (latency_ranges_hsplit): ``h_coeffs_fn() -> H tensor`` on the
    lead (witness map + NTT chain), ``bcast(tensor) -> done()`` the group broadcaster (group_broadcaster) -- the
    lead's tensor goes out, the others receive into ``h_coeffs_fn(None)``'s buffer -- and ``share_fn(ranges, h) ->
    576 bytes``.  The lead starts the broadcast and proves all its ranges with the H it computed while the
    broadcast is in flight; every other rank first proves its L / A / B slice (no H needed: it runs while the
    lead's NTT chain and the broadcast are under way), then waits for H and proves its H slice.  Returns a list of
    one or two shares (prove_partitions_balanced carries both)."""
    if k == 0:
        h = h_coeffs_fn()
        done = bcast(h)
        share = share_fn(ranges[0], h)
        done()
        return [share]
    rg = ranges[k]
    lab_only = [(rg[0][0], 0), rg[1], rg[2], rg[3]]
    h_only = [rg[0], (rg[1][0], 0), (rg[2][0], 0), (rg[3][0], 0)]
    first = share_fn(lab_only, None)
    h = bcast(h_coeffs_fn(None))()
    return [first, share_fn(h_only, h)]


def calibrate_hsplit(ctx, pk, circuit, z_dev: int, h_dev: int, reps: int = 1):
    """One GPU's times of the three parts of an H-split proof (after a warm call each): t_qap_ms (witness map + NTT
    chain, mi_groth16_h_coeffs_dev into h_dev), t_hmsm_ms (the whole H MSM from h_dev), t_lab_ms (L, A, B)."""
    import time

    from .core import h_coeffs_dev, prove_share_ranges

    sizes = (pk.n_h, pk.n_l, pk.n_a, pk.n_b)
    parts = {"t_qap_ms": lambda: h_coeffs_dev(ctx, circuit, z_dev, h_dev),
             "t_hmsm_ms": lambda: prove_share_ranges(ctx, pk, circuit, z_dev, [(0, sizes[0]), (0, 0), (0, 0), (0, 0)],
                                                     h_dev=h_dev),
             "t_lab_ms": lambda: prove_share_ranges(ctx, pk, circuit, z_dev,
                                                    [(0, 0), (0, sizes[1]), (0, sizes[2]), (0, sizes[3])])}
    t = {}
    for name, fn in parts.items():
        fn()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        ctx.synchronize()
        t[name] = 1e3 * (time.perf_counter() - t0) / reps
    return t


def lead_share_from_times(t_h: float, t_lab: float, group: int) -> float:
    """The lead rank's fraction of L, A and B that evens a group out: t_h = the H part alone (witness map, NTT
    chain, H MSM), t_lab = L, A and B alone, both on one GPU.  Lead: t_h + f t_lab; others: (1 - f) t_lab / (g - 1);
    equal at f = (t_lab - (g - 1) t_h) / (g t_lab), clamped to [0, 1] (0: H alone already outweighs a slice)."""
    if group <= 1 or t_lab <= 0:
        return 1.0
    return min(1.0, max(0.0, (t_lab - (group - 1) * t_h) / (group * t_lab)))


def calibrate_lead_share(ctx, pk, circuit, z, group: int, reps: int = 1):
    """Times the two halves of one proof on this GPU (after one warm call each) and returns
    (lead_share_from_times, {"t_h_ms", "t_lab_ms"}).  z: host bytes or a device pointer."""
    import time

    from .core import prove_share_ranges

    sizes = (pk.n_h, pk.n_l, pk.n_a, pk.n_b)
    h_only = [(0, sizes[0]), (0, 0), (0, 0), (0, 0)]
    lab = [(0, 0), (0, sizes[1]), (0, sizes[2]), (0, sizes[3])]
    t = {}
    for name, rg in (("t_h_ms", h_only), ("t_lab_ms", lab)):
        prove_share_ranges(ctx, pk, circuit, z, rg)
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            prove_share_ranges(ctx, pk, circuit, z, rg)
        ctx.synchronize()
        t[name] = 1e3 * (time.perf_counter() - t0) / reps
    return lead_share_from_times(t["t_h_ms"], t["t_lab_ms"], group), t


def agree_float(x, rank: int, device="cpu") -> float:
    """rank 0's value of x on every rank (one broadcast); x itself without a process group"""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    t = torch.tensor([float(x) if rank == 0 else 0.0], dtype=torch.float64).to(device)
    dist.broadcast(t, 0)
    return float(t.cpu().item())


def gather_shares(share: bytes, world: int, device="cpu"):
    """All-gather one MI_SHARE_BYTES record per rank (the latency mode's only exchange, 576 B per GPU)."""
    import torch

    if len(share) != SHARE_BYTES:
        raise ValueError(f"shares are {SHARE_BYTES} bytes")
    t = torch.from_numpy(np.frombuffer(share, dtype=np.uint8).copy()).to(device)
    return [b.tobytes() for b in _all_gather(t, world)]


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
_POINT_BYTES = {"vk": 1, "ic": 96, "h": 96, "l": 96, "a": 96, "b_g1": 96, "b_g2": 192}


def _broadcast_chunks(sizes, rank, src, device, chunk_bytes, source, sink, relay=False):
    """Broadcast every part of ``sizes`` (name -> bytes) from ``src`` in chunks of whole points of at most
    ``chunk_bytes``: ``source(name, offset, nbytes) -> uint8 tensor on device`` on the source rank,
    ``sink(name, offset, tensor)`` on the others (relay: the one rank of a world of one does both, the
    broadcast tensor going to its own sink).  Only one chunk is in flight per rank."""
    import torch
    import torch.distributed as dist

    is_src = relay or rank == src
    for k, n in sizes:
        esz = _POINT_BYTES[k]
        step = max(esz, chunk_bytes // esz * esz)
        for off in range(0, n, step):
            m = min(step, n - off)
            t = source(k, off, m) if is_src else torch.empty(m, dtype=torch.uint8, device=device)
            dist.broadcast(t, src)
            if relay or rank != src:
                sink(k, off, t)


def _broadcast_sizes(sizes, rank, src, device):
    import torch
    import torch.distributed as dist

    t = torch.tensor(sizes if rank == src else [0] * len(SRS_PARTS), dtype=torch.int64).to(device)
    dist.broadcast(t, src)
    return [int(x) for x in t.cpu().tolist()]


def broadcast_srs_parts(parts, rank: int, world: int, src: int = 0, device="cpu", chunk_bytes: int = 1 << 30):
    """Broadcast a proving key in the bellman wire layout (dict of SRS_PARTS -> bytes, held by ``src``) to
    every rank: one size vector, then each part in chunks of whole points (bounded staging memory).  The
    source returns its own dict untouched; a receiver assembles each part in ONE preallocated bytearray
    (no second copy).  For a device-resident key use broadcast_proving_key, which streams the chunks
    device to device and never materialises the key in host memory."""
    if world == 1:
        return dict(parts)
    sizes = _broadcast_sizes([len(parts[k]) for k in SRS_PARTS] if rank == src else None, rank, src, device)
    if rank == src:
        import torch

        views = {k: memoryview(parts[k]) for k in SRS_PARTS}
        source = (lambda k, off, m: torch.frombuffer(bytearray(views[k][off:off + m]), dtype=torch.uint8)
                  .to(device))
        _broadcast_chunks(list(zip(SRS_PARTS, sizes)), rank, src, device, chunk_bytes, source, None)
        return parts
    out = {k: bytearray(n) for k, n in zip(SRS_PARTS, sizes)}

    def sink(k, off, t):
        out[k][off:off + t.numel()] = memoryview(t.cpu().numpy())

    _broadcast_chunks(list(zip(SRS_PARTS, sizes)), rank, src, device, chunk_bytes, None, sink)
    return out


def broadcast_proving_key(ctx, pk, circuit, rank: int, world: int, src: int = 0, device="cpu", checked=False,
                          chunk_bytes: int = 1 << 30, self_relay: bool = False):
    """Rank ``src`` holds ``pk`` (e.g. ProvingKey.load_params from a v28 file); every other rank receives the
    key over the process group and loads it into its own GPU through the streaming loader
    (mi_srs_stream_*), chunk by chunk with the same rules as mi_srs_load (``checked``: subgroup checks).
    The reference reads the params file in every process (get_groth_params,
    core/parameter_cache.hpp:185-200); here one rank reads it and the others receive it.

    With backend "nccl" (``device`` a CUDA device) the source encodes each chunk on its GPU
    (mi_srs_export_query_dev), RCCL moves it over xGMI, and the receiver decodes it in place from device
    memory: no rank holds the key in host memory.  With gloo the chunks travel through host tensors, one
    chunk at a time.  Memory per rank beyond the key itself: one chunk.  Returns this rank's ProvingKey.

    ``self_relay`` (a world of one with an initialised group): the one rank is source and receiver, every
    chunk goes through the group's broadcast and is decoded into a second key, which is returned.  That
    runs the whole device path -- export, RCCL broadcast, on-device decode -- on a one-GPU box."""
    import torch

    from .core import ProvingKey

    relay = bool(self_relay) and world == 1
    if world == 1 and not relay:
        return pk
    if relay and not _group_active(1):
        raise RuntimeError("self_relay needs an initialised process group")
    is_src, is_dst = (True, True) if relay else (rank == src, rank != src)
    on_gpu = torch.device(device).type == "cuda"
    sizes = None
    if is_src:
        vk, ic = pk.verifying_key()
        sizes = [len(vk), len(ic), 96 * pk.n_h, 96 * pk.n_l, 96 * pk.n_a, 96 * pk.n_b, 192 * pk.n_b]
    sizes = _broadcast_sizes(sizes, rank, src, device)
    small_src = {"vk": vk, "ic": ic} if is_src else None
    small = {"vk": bytearray(sizes[0]), "ic": bytearray(sizes[1])}
    gpu = torch.device("cuda", ctx.device) if hasattr(ctx, "device") else torch.device("cuda")

    def source_small(k, off, m):
        return torch.frombuffer(bytearray(small_src[k][off:off + m]), dtype=torch.uint8).to(device)

    def sink_small(k, off, t):
        small[k][off:off + t.numel()] = memoryview(t.cpu().numpy())

    which = {k: i for i, k in enumerate(SRS_PARTS[2:])}

    def source(k, off, m):
        t = torch.empty(m, dtype=torch.uint8, device=gpu)
        # the library writes t on its own stream: torch's stream must be done with this memory first
        torch.cuda.current_stream(gpu).synchronize()
        pk.export_query_dev(which[k], off // _POINT_BYTES[k], m // _POINT_BYTES[k], t.data_ptr())
        return t if on_gpu else t.cpu()

    _broadcast_chunks([("vk", sizes[0]), ("ic", sizes[1])], rank, src, device, chunk_bytes,
                      source_small if is_src else None, sink_small if is_dst else None, relay)
    queries = list(zip(SRS_PARTS[2:], sizes[2:]))
    if not is_dst:
        _broadcast_chunks(queries, rank, src, device, chunk_bytes, source, None)
        return pk
    counts = [n // _POINT_BYTES[k] for k, n in queries]
    stream = ProvingKey.stream_begin(ctx, circuit, bytes(small["vk"]), bytes(small["ic"]), counts, checked)

    def sink(k, off, t):
        if t.is_cuda:
            torch.cuda.current_stream(t.device).synchronize()  # the broadcast landed before the decode reads it
            stream.part(which[k], off // _POINT_BYTES[k], t.data_ptr(), t.numel() // _POINT_BYTES[k], on_device=True)
        else:
            stream.part(which[k], off // _POINT_BYTES[k], t.numpy(), t.numel() // _POINT_BYTES[k], on_device=False)

    try:
        _broadcast_chunks(queries, rank, src, device, chunk_bytes, source if relay else None, sink, relay)
    except BaseException:
        stream.abort()
        raise
    return stream.end()
