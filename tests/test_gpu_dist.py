"""GPU: the multi-GPU entry points as the driver runs them, on this pool's one-GPU boxes.

* `bench.py --gpus 2` with no launcher: the parent starts two rank processes itself (bench.spawn_ranks), before
  any GPU call, and forwards rank 0's JSON line.  Both ranks share device 0 and gloo carries the collectives
  (MI_BENCH_SHARED_DEVICE / MI_BENCH_BACKEND: RCCL refuses two ranks on one device); the line must report
  n_gpus 2 and a config-5 leg (3 Window-PoSt partitions of 8 sectors: 0 and 1 whole, 2 split over both ranks)
  whose every proof pairing-verifies.  That is the shape of the driver's 8-GPU command (10 partitions of the
  real 2349-sector circuit; SURVEY 8(e), api/post.hpp:305-348, src/api/post.cpp:37-46).
* The RCCL path itself: a world of one over backend "nccl" on device tensors -- gather_multiproof,
  gather_shares, agree_blinding, and broadcast_proving_key in self-relay (export on the GPU, RCCL broadcast,
  on-device decode into a second key); the relayed key proves the oracle's bytes.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def test_bench_gpus2_spawns_ranks_and_measures_config5():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(MI_BENCH_BACKEND="gloo", MI_BENCH_SHARED_DEVICE="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--log-rows", "12", "--msm-reps", "1", "--no-cpu-baseline", "--no-device-resident", "--tree-log-nodes", "0",
           "--sdr-log-labels", "0", "--config4-log-rows", "0", "--stacked-log-nodes", "0", "--winning-log-nodes", "0",
           "--post-sectors", "8", "--post-log-nodes", "12", "--post-partitions", "3"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=240)
    err = r.stderr.decode()[-3000:]
    assert r.returncode == 0, err
    lines = [ln for ln in r.stdout.decode().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout.decode()[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["verified"] and out["verified_proofs"] == 2 * 2
    c5 = out["config5"]
    assert c5 and "error" not in c5, c5
    assert c5["n_gpus"] == 2 and c5["partitions"] == 3 and c5["verified"] and c5["verified_proofs"] == 3
    assert c5["split_partitions"] == [{"partition": 2, "ranks": [0, 1]}]


def test_bench_refuses_launcher_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env, cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert r.returncode != 0 and b"must agree" in r.stderr


def _nccl_worker(rank, port, outdir):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "crypto3-fil-proofs_amd"), os.path.join(root, "tests", "golden")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import circuits
    import fil_groth16 as fg
    from fil_groth16.core import FR_MODULUS
    from fil_groth16.distributed import agree_blinding, broadcast_proving_key, gather_multiproof, gather_shares

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    dev = torch.device("cuda", 0)
    c = fg.Context(0)
    n_in, n_aux, rws, z = circuits.random_circuit(91, 1200, n_in=4, n_free=24)
    gc = fg.Circuit(c, len(rws), n_in, n_aux, circuits.to_csr(rws))
    pk = fg.generate_random_parameters(c, gc, circuits.toxic())
    zb = circuits.z_bytes(z)
    proofs = fg.prove_batch(c, pk, gc, [zb, zb], [(3, 4), (5, 6)])
    mp_ = gather_multiproof(proofs, 2, 0, 1, dev)
    share = fg.prove_share(c, pk, gc, zb, 0, 1)
    sh = gather_shares(share, 1, dev)
    bl = agree_blinding(3, 0, dev)
    # several chunks per query: chunk_bytes of 64 G1 points
    pk2 = broadcast_proving_key(c, pk, gc, 0, 1, device=dev, checked=True, chunk_bytes=96 * 64, self_relay=True)
    p2 = fg.prove(c, pk2, gc, zb, 3, 4)
    assert pk2.verifying_key() == pk.verifying_key()
    res = {"multiproof": mp_.hex(), "proofs": [p.hex() for p in proofs], "shares_equal": sh == [share],
           "blinding_ok": len(bl) == 3 and all(0 <= x < FR_MODULUS for pr in bl for x in pr) and
           len({x for pr in bl for x in pr}) == 6, "relayed_proof": p2.hex(), "backend": dist.get_backend()}
    with open(os.path.join(outdir, "nccl.json"), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()
    del pk, pk2, gc
    c.close()


def test_nccl_world1_collectives_on_device_tensors(oracle, tmp_path):
    import circuits
    import torch.multiprocessing as mp

    mp.spawn(_nccl_worker, args=(_free_port(), str(tmp_path)), nprocs=1, join=True)
    res = json.load(open(tmp_path / "nccl.json"))
    n_in, n_aux, rws, z = circuits.random_circuit(91, 1200, n_in=4, n_free=24)
    op = oracle.OracleParams(oracle.OracleCircuit(len(rws), n_in, n_aux, circuits.to_csr(rws)), circuits.toxic())
    zb = circuits.z_bytes(z)
    want = [op.prove(zb, 3, 4)[0], op.prove(zb, 5, 6)[0]]
    assert res["backend"] == "nccl"
    assert [bytes.fromhex(p) for p in res["proofs"]] == want
    assert bytes.fromhex(res["multiproof"]) == b"".join(want)
    assert res["shares_equal"] and res["blinding_ok"]
    assert bytes.fromhex(res["relayed_proof"]) == want[0]
