"""CPU: the N>1 path (one process per device, partition sharding, proof gather) with gloo,
world_size 2.  Proofs are produced by the oracle here (CPU); on GPUs the same code runs with
backend "nccl" (RCCL) and the HIP prover (bench.py)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, num_partitions, outdir):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "crypto3-fil-proofs_amd"), os.path.join(root, "oracle"),
              os.path.join(root, "tests", "golden")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import circuits
    import oracle_py
    from fil_groth16.compound import shard_partitions
    from fil_groth16.distributed import gather_multiproof

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_in, n_aux, rows, z = circuits.random_circuit(61, 40)
    oc = oracle_py.OracleCircuit(len(rows), n_in, n_aux, circuits.to_csr(rows))
    P = oracle_py.OracleParams(oc, circuits.toxic())
    zb = circuits.z_bytes(z)
    mine = shard_partitions(num_partitions, rank, world)
    local = [P.prove(zb, 100 + p, 200 + p)[0] for p in mine]  # partition p uses blinding (100+p, 200+p)
    mp_bytes = gather_multiproof(local, num_partitions, rank, world)
    with open(os.path.join(outdir, f"r{rank}.bin"), "wb") as f:
        f.write(mp_bytes)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("num_partitions", [3, 4])
def test_gloo_world2_gather(tmp_path, oracle, num_partitions):
    import circuits

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), num_partitions, str(tmp_path)), nprocs=world, join=True)
    outs = [open(tmp_path / f"r{r}.bin", "rb").read() for r in range(world)]
    assert outs[0] == outs[1]
    # serial reference: compound_proof::circuit_proofs order
    n_in, n_aux, rows, z = circuits.random_circuit(61, 40)
    oc = oracle.OracleCircuit(len(rows), n_in, n_aux, circuits.to_csr(rows))
    P = oracle.OracleParams(oc, circuits.toxic())
    zb = circuits.z_bytes(z)
    serial = b"".join(P.prove(zb, 100 + p, 200 + p)[0] for p in range(num_partitions))
    assert outs[0] == serial


def _split_worker(rank, world, port, outdir):
    """Latency mode over gloo: rank k's share (oracle MSMs over its slices), all-gather, host assembly
    through the C ABI (mi_groth16_assemble needs no device)."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "crypto3-fil-proofs_amd"), os.path.join(root, "oracle"),
              os.path.join(root, "tests", "golden"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import circuits
    import fil_groth16 as fg
    import oracle_py
    import split_oracle
    from fil_groth16.distributed import gather_shares

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_in, n_aux, rows, z = circuits.random_circuit(71, 60)
    mats = circuits.to_csr(rows)
    P = oracle_py.OracleParams(oracle_py.OracleCircuit(len(rows), n_in, n_aux, mats), circuits.toxic())
    mine = split_oracle.shares(oracle_py, P, n_in, n_aux, mats, circuits.z_bytes(z), world)[rank]
    shares = gather_shares(mine, world)
    proof = fg.assemble(P.export()["vk"], shares, 17, 19)
    with open(os.path.join(outdir, f"s{rank}.bin"), "wb") as f:
        f.write(proof)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_split_proof(tmp_path, oracle):
    """SURVEY.md 8e single-proof latency mode: two ranks' shares, one all-gather, the same proof bytes
    on both ranks as the serial prove."""
    import circuits

    world = 2
    mp.spawn(_split_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    outs = [open(tmp_path / f"s{r}.bin", "rb").read() for r in range(world)]
    n_in, n_aux, rows, z = circuits.random_circuit(71, 60)
    P = oracle.OracleParams(oracle.OracleCircuit(len(rows), n_in, n_aux, circuits.to_csr(rows)), circuits.toxic())
    assert outs[0] == outs[1] == P.prove(circuits.z_bytes(z), 17, 19)[0]


def _partitions_worker(rank, world, port, num_partitions, outdir):
    """bench.py --partitions P, with the oracle standing in for the GPU prover: the same runner
    (fil_groth16.distributed.prove_partitions) and gather over gloo instead of RCCL."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "crypto3-fil-proofs_amd"), os.path.join(root, "oracle"),
              os.path.join(root, "tests", "golden")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import circuits
    import oracle_py
    from fil_groth16.distributed import prove_partitions

    oracle_py.set_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_in, n_aux, rows, z = circuits.random_circuit(62, 40)
    P = oracle_py.OracleParams(oracle_py.OracleCircuit(len(rows), n_in, n_aux, circuits.to_csr(rows)),
                               circuits.toxic())
    zb = circuits.z_bytes(z)
    proven = []

    def prove_fn(ids):
        proven.extend(ids)
        return [P.prove(zb, 300 + p, 400 + p)[0] for p in ids]

    buf = prove_partitions(prove_fn, num_partitions, rank, world)
    with open(os.path.join(outdir, f"p{rank}.bin"), "wb") as f:
        f.write(buf)
    with open(os.path.join(outdir, f"ids{rank}.txt"), "w") as f:
        f.write(",".join(map(str, proven)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,num_partitions", [(2, 10), (8, 10), (3, 2)])
def test_gloo_partition_runner(tmp_path, oracle, world, num_partitions):
    """Config 5 shape: 10 Window-PoSt partitions over 8 ranks (two rounds on ranks 0 and 1), and fewer
    partitions than ranks; every rank ends with the serial multi-proof."""
    import circuits

    mp.spawn(_partitions_worker, args=(world, _free_port(), num_partitions, str(tmp_path)), nprocs=world,
             join=True)
    outs = [open(tmp_path / f"p{r}.bin", "rb").read() for r in range(world)]
    ids = [open(tmp_path / f"ids{r}.txt").read() for r in range(world)]
    assert ids == [",".join(map(str, range(r, num_partitions, world))) for r in range(world)]
    n_in, n_aux, rows, z = circuits.random_circuit(62, 40)
    P = oracle.OracleParams(oracle.OracleCircuit(len(rows), n_in, n_aux, circuits.to_csr(rows)), circuits.toxic())
    zb = circuits.z_bytes(z)
    serial = b"".join(P.prove(zb, 300 + p, 400 + p)[0] for p in range(num_partitions))
    assert all(o == serial for o in outs)


def test_balanced_schedule():
    """Config 5 on 8 GPUs: partitions 0-7 whole, 8 and 9 each over a group of four ranks; every partition
    exactly once, every rank in at most one group, groups of one collapse into whole proofs."""
    from fil_groth16.distributed import balanced_schedule

    whole, tail = balanced_schedule(10, 8)
    assert whole == [[r] for r in range(8)]
    assert tail == [(8, [0, 1, 2, 3]), (9, [4, 5, 6, 7])]
    assert balanced_schedule(10, 4) == ([[0, 4], [1, 5], [2, 6], [3, 7]], [(8, [0, 1]), (9, [2, 3])])
    assert balanced_schedule(10, 2) == ([[0, 2, 4, 6, 8], [1, 3, 5, 7, 9]], [])
    assert balanced_schedule(3, 2) == ([[0], [1]], [(2, [0, 1])])
    assert balanced_schedule(2, 3) == ([[], [], [1]], [(0, [0, 1])])  # groups [0, 1] and [2]: rank 2 proves 1 whole
    for P in range(0, 13):
        for W in range(1, 9):
            whole, tail = balanced_schedule(P, W)
            ids = sorted([p for w in whole for p in w] + [p for p, _ in tail])
            assert ids == list(range(P))
            grouped = [r for _, rs in tail for r in rs]
            assert len(grouped) == len(set(grouped)) and all(len(rs) > 1 for _, rs in tail)
            # makespan in units of one whole proof: never worse than round-robin
            assert max(len(w) for w in whole) <= -(-P // W)


def _balanced_worker(rank, world, port, num_partitions, outdir):
    """The balanced config-5 runner with the oracle standing in for the GPU prover: whole partitions by the
    oracle prove, tail partitions by oracle shares (split_oracle) assembled through the C ABI."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "crypto3-fil-proofs_amd"), os.path.join(root, "oracle"),
              os.path.join(root, "tests", "golden"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import circuits
    import fil_groth16 as fg
    import oracle_py
    import split_oracle
    from fil_groth16.distributed import agree_blinding, prove_partitions_balanced

    oracle_py.set_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_in, n_aux, rows, z = circuits.random_circuit(63, 40)
    mats = circuits.to_csr(rows)
    P = oracle_py.OracleParams(oracle_py.OracleCircuit(len(rows), n_in, n_aux, mats), circuits.toxic())
    zb = circuits.z_bytes(z)
    vk = P.export()["vk"]
    log = []

    def prove_fn(ids):
        log.extend(("whole", p) for p in ids)
        return [P.prove(zb, 300 + p, 400 + p)[0] for p in ids]

    def share_fn(p, k, g):
        log.append(("share", p, k, g))
        return split_oracle.shares(oracle_py, P, n_in, n_aux, mats, zb, g)[k]

    buf = prove_partitions_balanced(prove_fn, share_fn, lambda p, sh: fg.assemble(vk, sh, 300 + p, 400 + p),
                                    num_partitions, rank, world)
    rs = agree_blinding(2, rank)
    with open(os.path.join(outdir, f"b{rank}.bin"), "wb") as f:
        f.write(buf)
    with open(os.path.join(outdir, f"log{rank}.txt"), "w") as f:
        f.write(repr(log) + "\n" + repr(rs))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,num_partitions", [(2, 3), (3, 5), (4, 2)])
def test_gloo_balanced_runner(tmp_path, oracle, world, num_partitions):
    """Tail partitions split over rank groups (latency-mode shares + host assembly) give the same multi-proof
    bytes as the serial prove on every rank; the blinding rank 0 draws reaches every rank unchanged."""
    import circuits
    from fil_groth16.distributed import balanced_schedule

    mp.spawn(_balanced_worker, args=(world, _free_port(), num_partitions, str(tmp_path)), nprocs=world, join=True)
    outs = [open(tmp_path / f"b{r}.bin", "rb").read() for r in range(world)]
    logs = [open(tmp_path / f"log{r}.txt").read().split("\n") for r in range(world)]
    whole, tail = balanced_schedule(num_partitions, world)
    assert tail, "the case must exercise a split partition"
    for r in range(world):
        exp = [("whole", p) for p in whole[r]] + [("share", p, rs.index(r), len(rs)) for p, rs in tail if r in rs]
        assert logs[r][0] == repr(exp)
    assert len({l[1] for l in logs}) == 1  # agree_blinding: identical pairs on every rank
    n_in, n_aux, rows, z = circuits.random_circuit(63, 40)
    P = oracle.OracleParams(oracle.OracleCircuit(len(rows), n_in, n_aux, circuits.to_csr(rows)), circuits.toxic())
    zb = circuits.z_bytes(z)
    serial = b"".join(P.prove(zb, 300 + p, 400 + p)[0] for p in range(num_partitions))
    assert all(o == serial for o in outs)


def _srs_worker(rank, world, port, outdir):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "crypto3-fil-proofs_amd"), os.path.join(root, "oracle"),
              os.path.join(root, "tests", "golden")):
        sys.path.insert(0, p)
    import hashlib

    import torch.distributed as dist

    import circuits
    import oracle_py
    from fil_groth16.distributed import SRS_PARTS, broadcast_srs_parts

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    parts = None
    if rank == 1:  # a non-zero source rank, and chunks far smaller than the parts
        n_in, n_aux, rows, z = circuits.random_circuit(63, 40)
        oc = oracle_py.OracleCircuit(len(rows), n_in, n_aux, circuits.to_csr(rows))
        parts = oracle_py.OracleParams(oc, circuits.toxic()).export()
    got = broadcast_srs_parts(parts, rank, world, src=1, chunk_bytes=1000)
    with open(os.path.join(outdir, f"s{rank}.txt"), "w") as f:
        f.write(",".join(hashlib.sha256(got[k]).hexdigest() for k in SRS_PARTS))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_srs_broadcast(tmp_path):
    """One rank holds the proving key (bellman wire layout); every rank ends with identical bytes."""
    import hashlib

    import circuits
    import oracle_py
    from fil_groth16.distributed import SRS_PARTS

    world = 3
    mp.spawn(_srs_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    outs = [open(tmp_path / f"s{r}.txt").read() for r in range(world)]
    n_in, n_aux, rows, z = circuits.random_circuit(63, 40)
    oc = oracle_py.OracleCircuit(len(rows), n_in, n_aux, circuits.to_csr(rows))
    ex = oracle_py.OracleParams(oc, circuits.toxic()).export()
    assert all(len(ex[k]) > 1000 or k == "vk" for k in ("h", "l", "a", "b_g2"))
    exp = ",".join(hashlib.sha256(bytes(ex[k])).hexdigest() for k in SRS_PARTS)
    assert outs == [exp] * world


# ------------------------------------------------------------------ latency groups that compute H once
@pytest.mark.parametrize("g", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("lead", [0.0, 0.146, 0.5, 1.0])
def test_latency_ranges_partition_every_query(g, lead):
    """Rank 0 of a group takes the whole H query (it alone runs the witness map + NTT chain) and `lead` of L, A,
    B; the others split the rest: every query is covered exactly once, in contiguous order."""
    from fil_groth16.distributed import latency_ranges

    sizes = (1023, 1000, 977, 501)
    rg = latency_ranges(sizes, g, lead)
    assert len(rg) == g
    for q, n in enumerate(sizes):
        pos = 0
        for k in range(g):
            lo, cnt = rg[k][q]
            assert lo == pos and cnt >= 0
            pos += cnt
        assert pos == n
    assert rg[0][0] == (0, sizes[0]) and all(rg[k][0][1] == 0 for k in range(1, g))
    if g > 1:
        counts = [rg[k][1][1] for k in range(1, g)]
        assert max(counts) - min(counts) <= 1


def test_lead_share_from_times():
    from fil_groth16.distributed import lead_share_from_times

    assert lead_share_from_times(467.0, 1284.0, 4) == 0.0  # H alone outweighs a third of L/A/B
    f = lead_share_from_times(467.0, 1284.0, 2)
    assert abs((467.0 + f * 1284.0) - (1 - f) * 1284.0) < 1e-6
    assert lead_share_from_times(0.0, 100.0, 4) == 0.25 and lead_share_from_times(5.0, 100.0, 1) == 1.0


def _ranges_worker(rank, world, port, outdir):
    """The balanced runner whose tail groups use latency_ranges (H once per group), oracle range shares."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "crypto3-fil-proofs_amd"), os.path.join(root, "oracle"),
              os.path.join(root, "tests", "golden"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import circuits
    import fil_groth16 as fg
    import oracle_py
    import split_oracle
    from fil_groth16.distributed import agree_float, latency_ranges, prove_partitions_balanced

    oracle_py.set_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_in, n_aux, rows, z = circuits.random_circuit(64, 40)
    mats = circuits.to_csr(rows)
    P = oracle_py.OracleParams(oracle_py.OracleCircuit(len(rows), n_in, n_aux, mats), circuits.toxic())
    zb = circuits.z_bytes(z)
    ex = P.export()
    idx_a, idx_b = split_oracle.densities(n_in, n_aux, mats)
    sizes = (P.d - 1, n_aux, len(idx_a), len(idx_b))
    lead = agree_float(0.3 if rank == 0 else 0.9, rank)  # rank 0's value reaches every rank

    def share_fn(p, k, g):
        rg = latency_ranges(sizes, g, lead)
        return split_oracle.shares_ranges(oracle_py, P, n_in, n_aux, mats, zb, [rg[k]])[0]

    buf = prove_partitions_balanced(lambda ids: [P.prove(zb, 300 + p, 400 + p)[0] for p in ids], share_fn,
                                    lambda p, sh: fg.assemble(ex["vk"], sh, 300 + p, 400 + p), 5, rank, world)
    with open(os.path.join(outdir, f"r{rank}.bin"), "wb") as f:
        f.write(buf + repr(lead).encode())
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_balanced_runner_h_once(tmp_path, oracle):
    """5 partitions over 3 ranks: 3 whole, 2 tail partitions over groups whose lead rank alone computes H; the
    multi-proof equals the serial one on every rank."""
    import circuits

    mp.spawn(_ranges_worker, args=(3, _free_port(), str(tmp_path)), nprocs=3, join=True)
    n_in, n_aux, rows, z = circuits.random_circuit(64, 40)
    P = oracle.OracleParams(oracle.OracleCircuit(len(rows), n_in, n_aux, circuits.to_csr(rows)), circuits.toxic())
    zb = circuits.z_bytes(z)
    serial = b"".join(P.prove(zb, 300 + p, 400 + p)[0] for p in range(5)) + repr(0.3).encode()
    assert all(open(tmp_path / f"r{r}.bin", "rb").read() == serial for r in range(3))


# ------------------------------------------------------------------ latency groups that compute H once and split it
@pytest.mark.parametrize("g", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("h_lead,lab_lead", [(0.0, 0.0), (0.69, 0.0), (1.0, 0.3), (1.0, 1.0)])
def test_latency_ranges_hsplit_partition_every_query(g, h_lead, lab_lead):
    from fil_groth16.distributed import latency_ranges_hsplit

    sizes = (1023, 1000, 977, 501)
    rg = latency_ranges_hsplit(sizes, g, h_lead, lab_lead)
    assert len(rg) == g
    for q, n in enumerate(sizes):
        pos = 0
        for k in range(g):
            lo, cnt = rg[k][q]
            assert lo == pos and cnt >= 0
            pos += cnt
        assert pos == n
        if g > 1:
            counts = [rg[k][q][1] for k in range(1, g)]
            assert max(counts) - min(counts) <= 1


def test_hsplit_fractions_even_the_group():
    """Window-PoSt numbers of round 4 (t_qap 202 ms, H MSM 283 ms, L/A/B 1,104 ms): four ranks finish together at
    ~(t_qap + t_hmsm + t_lab) / 4 instead of the lead's 571 ms with H unsplit."""
    from fil_groth16.distributed import hsplit_fractions

    t_qap, t_h, t_lab = 202.0, 283.0, 1104.0
    for g in (2, 3, 4, 8):
        h, f = hsplit_fractions(t_qap, t_h, t_lab, g)
        lead = t_qap + h * t_h + f * t_lab
        other = ((1 - h) * t_h + (1 - f) * t_lab) / (g - 1)
        if 0.0 < h < 1.0 or 0.0 < f < 1.0:
            assert abs(lead - other) < 1e-6
        assert max(lead, other) <= 1.0001 * max(t_qap, (t_qap + t_h + t_lab) / g)
    h, f = hsplit_fractions(t_qap, t_h, t_lab, 4)
    assert 0.68 < h < 0.70 and f == 0.0
    assert hsplit_fractions(500.0, 10.0, 100.0, 4) == (0.0, 0.0)  # the NTT chain alone outweighs a share
    assert hsplit_fractions(1.0, 10.0, 1000.0, 2)[0] == 1.0  # small H: the lead also takes L/A/B
    assert hsplit_fractions(1.0, 1.0, 1.0, 1) == (1.0, 1.0)


def _hsplit_worker(rank, world, port, num_partitions, outdir):
    """The balanced runner with H-split tail groups: the lead's H coefficients (oracle, device order) are broadcast
    over the group's subgroup; the others prove L/A/B first, then their H slice from the received coefficients."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "crypto3-fil-proofs_amd"), os.path.join(root, "oracle"),
              os.path.join(root, "tests", "golden"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import numpy as np
    import torch
    import torch.distributed as dist

    import circuits
    import fil_groth16 as fg
    import oracle_py
    import split_oracle
    from fil_groth16.distributed import hsplit_fractions, hsplit_shares, latency_ranges_hsplit, \
        prove_partitions_balanced

    oracle_py.set_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_in, n_aux, rows, z = circuits.random_circuit(64, 40)
    mats = circuits.to_csr(rows)
    P = oracle_py.OracleParams(oracle_py.OracleCircuit(len(rows), n_in, n_aux, mats), circuits.toxic())
    zb = circuits.z_bytes(z)
    ex = P.export()
    idx_a, idx_b = split_oracle.densities(n_in, n_aux, mats)
    sizes = (P.d - 1, n_aux, len(idx_a), len(idx_b))
    used = {"h_from_bcast": 0}

    def share_fn(p, k, g, bcast):
        h_lead, lab_lead = hsplit_fractions(20.0, 30.0, 100.0, g)
        rg = latency_ranges_hsplit(sizes, g, h_lead, lab_lead)

        def h_coeffs(*arg):
            if arg and arg[0] is None:  # a receiver's buffer
                return torch.zeros(32 * P.d, dtype=torch.uint8)
            return torch.from_numpy(np.frombuffer(split_oracle.h_coeffs_perm(P, zb), dtype=np.uint8).copy())

        def one(ranges, h):
            if h is not None and k > 0:
                used["h_from_bcast"] += 1
            hp = h.numpy().tobytes() if h is not None else None
            return split_oracle.shares_ranges(oracle_py, P, n_in, n_aux, mats, zb, [ranges], hp)[0]

        return hsplit_shares(k, rg, h_coeffs, one, bcast)

    run = lambda: prove_partitions_balanced(lambda ids: [P.prove(zb, 300 + p, 400 + p)[0] for p in ids],  # noqa: E731
                                            share_fn, lambda p, sh: fg.assemble(ex["vk"], sh, 300 + p, 400 + p),
                                            num_partitions, rank, world, group_bcast=True)
    buf = run()
    from_bcast = used["h_from_bcast"]
    # the tail groups are created once per schedule, not per step, and freed by
    # destroy_group_broadcasters
    from fil_groth16 import distributed as fd

    groups = dict(fd._GROUPS)
    assert groups and run() == buf and fd._GROUPS == groups
    fd.destroy_group_broadcasters()
    assert not fd._GROUPS
    with open(os.path.join(outdir, f"r{rank}.bin"), "wb") as f:
        f.write(buf + repr(from_bcast).encode())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,num_partitions", [(4, 5), (3, 4)])
def test_gloo_balanced_runner_h_split(tmp_path, oracle, world, num_partitions):
    """One tail partition over a group of every rank, H computed once by the lead, broadcast over the group and
    split: the multi-proof equals the serial one on every rank, and every non-lead rank proved an H slice from the
    broadcast coefficients."""
    import circuits

    mp.spawn(_hsplit_worker, args=(world, _free_port(), num_partitions, str(tmp_path)), nprocs=world, join=True)
    n_in, n_aux, rows, z = circuits.random_circuit(64, 40)
    P = oracle.OracleParams(oracle.OracleCircuit(len(rows), n_in, n_aux, circuits.to_csr(rows)), circuits.toxic())
    zb = circuits.z_bytes(z)
    serial = b"".join(P.prove(zb, 300 + p, 400 + p)[0] for p in range(num_partitions))
    for r in range(world):
        got = open(tmp_path / f"r{r}.bin", "rb").read()
        assert got[:len(serial)] == serial
        assert int(got[len(serial):]) == (0 if r == 0 else 1)
