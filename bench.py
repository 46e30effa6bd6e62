#!/usr/bin/env python3
"""bench.py -- BASELINE metric: Groth16 constraints/sec (BLS12-381), plus MSM G1 Mpoints/s at 2^26.

Workload (BASELINE.json configs[2]): "Synthetic 2^26-constraint R1CS full Groth16 prove, 1 x MI355X".
A step = one full Groth16 prove of that circuit: witness map (R1CS evaluation), 7 NTTs, QAP
division, 4 G1 MSMs (H, L, A, B_G1) + 1 G2 MSM (B_G2) and proof assembly, proof bytes returned
to the host.  Inputs (witness, R1CS, proving key) are resident in HBM when the timed region
starts; the 192-byte proofs of all ranks are gathered to rank 0 over RCCL inside the timed region
(the MultiProof assembly of api/seal.hpp:306-308).

Multi-GPU: one process per GPU; each rank proves its own partition every step (PoSt / PoRep
partitions are independent proofs -- SURVEY.md §8e), so per-GPU work is fixed: weak scaling.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--log-rows 26]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "crypto3-fil-proofs_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# VALU bound of the accumulation kernel: v_mad_u64_u32 issue.  One wave64 MAD occupies its SIMD
# for 4 cycles: 1024 SIMDs x 64 lanes / 4 x 2.4 GHz = 39.3e12 lane-MADs/s.  (The dependent-chain
# microbench crypto3-fil-proofs_amd/microbench/madrate.hip sustains only 30.9e12 = 5.1 cycles,
# because each chain waits on its own previous MAD; the accumulation kernel's ISA -- 3920 MADs
# + ~1700 other VALU per mixed add, 14x29-bit limbs -- and its measured time imply the 4-cycle
# rate.)  One Fq multiplication = 392 MADs -> 100.3e9 Fq-mul/s of pure MAD issue; the remaining
# gap to it is the non-MAD instructions (carries, subtractions, selects).
MAD_RATE = 1024 * 64 / 4 * 2.4e9
FQ_MUL_MADS = 392
FQ_MUL_PER_MIXED_ADD = {"G1": 10, "G2": 28}  # madd-2008-s: 8M + 2S over Fq / Fq2 (Karatsuba 3M, 2M per sqr)
TOXIC_SEED = 0x5EED


def workload_name(log_rows):
    cfg = {26: " (BASELINE config 3)", 27: " (BASELINE config 4 shape: 32 GiB PoRep-sized, d = 2^27)"}
    return f"synthetic 2^{log_rows}-constraint R1CS full Groth16 prove" + cfg.get(log_rows, "")


def splitmix_frs(seed, n):
    out = []
    s = seed & 0xFFFFFFFFFFFFFFFF
    R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    for _ in range(n):
        v = 0
        for i in range(4):
            s = (s + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
            z = s
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
            v |= (z ^ (z >> 31)) << (64 * i)
        out.append(v % R)
    return out


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def cpu_baseline(args, fg, synth_mod, ctx):
    """The oracle (oracle/, a CPU restatement of the same prover) on a bounded sample of the same
    workload family: a 2^cpu_log_rows-constraint synthetic circuit, params generated on the GPU
    and exported, witness in host memory -> proof, timed with OpenMP threads = OMP_NUM_THREADS."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    oracle_py.set_threads(threads)
    sc = synth_mod.SynthCircuit(args.cpu_log_rows, args.n_in, args.seed)
    circ = sc.load(ctx)
    pk = fg.generate_random_parameters(ctx, circ, splitmix_frs(TOXIC_SEED, 5))
    vk, ic = pk.verifying_key()
    q = dict(h=pk.query(0), l=pk.query(1), a=pk.query(2), b_g1=pk.query(3), b_g2=pk.query(4), vk=vk, ic=ic)
    oc = oracle_py.OracleCircuit(sc.n, sc.n_in, sc.n_aux, sc.csr())
    op = oracle_py.OracleParams(oc, queries=q)
    zb = sc.z_bytes()
    r, s = splitmix_frs(77, 2)
    t0 = time.perf_counter()
    proof_cpu = op.prove(zb, r, s)[0]
    dt = time.perf_counter() - t0
    proof_gpu = fg.prove(ctx, pk, circ, zb, r, s)
    return {
        "value": sc.n / dt,
        "unit": "constraints/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle prove of the 2^{args.cpu_log_rows}-row synthetic circuit ({sc.n} constraints), "
                  f"{dt:.2f} s with {threads} OpenMP threads; GPU proof bytes identical: {proof_cpu == proof_gpu}",
        "seconds": dt,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--log-rows", type=int, default=26, help="log2 of the evaluation domain (config 3: 26)")
    ap.add_argument("--n-in", type=int, default=4)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--msm-reps", type=int, default=3, help="reps of the standalone 2^log-rows G1 MSM")
    ap.add_argument("--cpu-log-rows", type=int, default=21)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stats-json", default=None, help="write per-kernel timers here")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")
    device = torch.device("cuda", local_rank)

    import fil_groth16 as fg
    from fil_groth16 import synth as synth_mod

    t_setup = time.perf_counter()
    ctx = fg.Context(local_rank)
    sc = synth_mod.SynthCircuit(args.log_rows, args.n_in, args.seed)
    t_synth = time.perf_counter() - t_setup
    circ = sc.load(ctx)
    t_load = time.perf_counter() - t_setup - t_synth
    pk = fg.generate_random_parameters(ctx, circ, splitmix_frs(TOXIC_SEED, 5))
    ctx.synchronize()
    t_srs = time.perf_counter() - t_setup - t_synth - t_load
    z = torch.from_numpy(sc.z_array().copy()).to(device)  # witness resident in HBM
    torch.cuda.synchronize()
    n = sc.n
    log(rank, f"setup: synth {t_synth:.1f}s circuit load {t_load:.1f}s srs gen {t_srs:.1f}s; n={n} d={circ.d} "
              f"|a|={circ.n_a} |b|={circ.n_b}")

    blind = splitmix_frs(1000 + rank, 2 * (args.warmup + args.steps))
    for w in range(args.warmup):
        fg.prove(ctx, pk, circ, z.data_ptr(), blind[2 * w], blind[2 * w + 1])
    ctx.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.reset_stats()

    t0 = time.perf_counter()
    proofs = []
    for k in range(args.steps):
        i = args.warmup + k
        proofs.append(fg.prove(ctx, pk, circ, z.data_ptr(), blind[2 * i], blind[2 * i + 1]))
    # MultiProof assembly: gather every rank's 192-byte proofs to rank 0 over RCCL
    local = torch.from_numpy(np.frombuffer(b"".join(proofs), dtype=np.uint8).copy()).to(device)
    if dist:
        bufs = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(bufs, local)
        gathered = torch.cat(bufs).cpu().numpy().tobytes() if rank == 0 else None
    else:
        gathered = local.cpu().numpy().tobytes()
    ctx.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    stats = ctx.stats()

    # secondary metric: standalone G1 MSM over the resident 2^log_rows - 1 h-query points
    msm_n = pk.n_h
    pts = pk.points(0)
    rng = np.random.default_rng(7 + rank)
    sw = rng.integers(0, 2**64, size=(msm_n, 4), dtype=np.uint64)
    sw[:, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)
    sc_dev = torch.from_numpy(sw.view(np.uint8).reshape(-1)).to(device)
    pts.msm_dev(sc_dev.data_ptr(), msm_n)  # warm
    ctx.synchronize()
    tm = time.perf_counter()
    for _ in range(args.msm_reps):
        pts.msm_dev(sc_dev.data_ptr(), msm_n)
    ctx.synchronize()
    msm_dt = (time.perf_counter() - tm) / args.msm_reps
    # BASELINE configs[1]: 2^20-point G1 MSM + 2^20-element Fr NTT (device-resident inputs)
    micro = {}
    if msm_n >= (1 << 20):
        m20 = 1 << 20
        pts.msm_dev(sc_dev.data_ptr(), m20)
        ctx.synchronize()
        tm = time.perf_counter()
        for _ in range(10):
            pts.msm_dev(sc_dev.data_ptr(), m20)
        ctx.synchronize()
        t20 = (time.perf_counter() - tm) / 10
        x = torch.from_numpy(sw[:m20].copy().view(np.uint8).reshape(-1)).to(device)
        ctx.ntt_dev(x.data_ptr(), 20, False, False)
        ctx.synchronize()
        tm = time.perf_counter()
        for _ in range(10):
            ctx.ntt_dev(x.data_ptr(), 20, False, False)
        ctx.synchronize()
        n20 = (time.perf_counter() - tm) / 10
        micro = {"workload": "BASELINE configs[1]: 2^20-point G1 MSM + 2^20-element Fr NTT, device-resident",
                 "msm_g1_2e20_ms": t20 * 1e3, "msm_g1_2e20_mpoints_per_s": m20 / t20 / 1e6,
                 "ntt_fr_2e20_ms": n20 * 1e3, "ntt_fr_2e20_melems_per_s": m20 / n20 / 1e6}
        del x
    del sc_dev

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args, fg, synth_mod, ctx)
        except Exception as e:  # reported, never fatal to the GPU measurement
            cpu = {"value": None, "unit": "constraints/s", "cores": None, "kind": "port", "sample": f"failed: {e}"}

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    # roofline of the dominant kernel (largest share of device time in the timed region)
    kernels = {
        "k_accum_level0<G1>": (stats["accum_g1"], 128.0, "G1"),
        "k_accum_level0<G2>": (stats["accum_g2"], 224.0, "G2"),
    }
    dom_name, (dom, bytes_per_unit, grp) = max(kernels.items(), key=lambda kv: kv[1][0]["ms"])
    avg_ms = dom["ms"] / max(dom["launches"], 1)
    units_per_launch = dom["units"] / max(dom["launches"], 1)
    achieved = bytes_per_unit * units_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else None
    # HBM traffic per launch from the committed rocprofv3 PMC summary of the same kernel/workload
    traffic, traffic_src = None, None
    prof_dir = os.path.join(ROOT, "profiles")
    if os.path.isdir(prof_dir):
        for fn in sorted(os.listdir(prof_dir), reverse=True):
            if fn.endswith("_summary.json"):
                try:
                    ps = json.load(open(os.path.join(prof_dir, fn)))
                    dk = ps.get("dominant_kernel", {})
                    if grp == "G1" and "hbm_bytes_per_point" in dk and ps.get("workload") == \
                            workload_name(args.log_rows):
                        traffic = dk["hbm_bytes_per_point"] * units_per_launch
                        traffic_src = fn
                        break
                except Exception:
                    pass
    # secondary (binding) roofline: Fq multiplications per second vs the MAD-issue bound, over the mixed
    # additions the accumulation actually issued (non-zero signed digits, counted by the library)
    madds_per_launch = dom.get("madds", 0) / max(dom["launches"], 1)
    fq_muls = madds_per_launch * FQ_MUL_PER_MIXED_ADD[grp]
    valu_ach = fq_muls / (avg_ms * 1e-3) if avg_ms > 0 and fq_muls else None
    valu_peak = MAD_RATE / FQ_MUL_MADS
    total_steps = args.steps * world
    value = n * total_steps / dt
    out = {
        "metric": "Groth16 constraints/sec (BLS12-381); MSM G1 Mpoints/s at 2^26",
        "value": value,
        "unit": "constraints/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 limbs (Fq 381-bit / Fr 255-bit Montgomery)",
        "data": "synthetic R1CS + satisfying witness (csrc/synth.hip), proving key generated on device from "
                "fixed toxic waste",
        "config": {"workload": workload_name(args.log_rows),
                   "constraints": n, "domain": circ.d, "num_inputs": sc.n_in, "num_aux": sc.n_aux,
                   "a_query": circ.n_a, "b_query": circ.n_b, "proofs_per_step": world,
                   "parallelism": f"partition-sharded x{world}"},
        "msm_g1_mpoints_per_s": msm_n / msm_dt / 1e6,
        "msm_g1_points": msm_n,
        "config2_micro": micro,
        "roofline": {
            "bound": "hbm",
            "kernel": dom_name,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS if achieved else None,
            "traffic": traffic,
            "traffic_source": f"profiles/{traffic_src} (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, per point x "
                              f"points per launch)" if traffic_src else None,
            "avg_launch_ms": avg_ms,
            "units_per_launch": units_per_launch,
            "algorithmic_bytes_per_unit": bytes_per_unit,
            "note": "VALU-integer-bound kernel (BLS12-381 Montgomery multiplications); HBM fraction is reported "
                    "per BASELINE.json north_star; the binding roofline is 'valu_roofline'",
        },
        "valu_roofline": {
            "bound": "valu (v_mad_u64_u32 issue)",
            "kernel": dom_name,
            "achieved": valu_ach,
            "peak": valu_peak,
            "unit": "Fq-mul/s",
            "frac": valu_ach / valu_peak if valu_ach else None,
            "madds_per_launch": madds_per_launch,
            "model": f"{FQ_MUL_PER_MIXED_ADD[grp]} Fq-mul per mixed add x mixed adds issued (non-zero signed digits "
                     f"counted by the library; split-mode MSMs: 2n half-scalar points over 6 windows); "
                     f"peak = v_mad_u64_u32 issue rate / {FQ_MUL_MADS} MADs",
        },
        "cpu_baseline": cpu,
        "timers_ms": {k: round(v["ms"], 3) for k, v in stats.items()},
        "setup_s": {"synth": t_synth, "circuit_load": t_load, "srs_generate": t_srs},
        "multiproof_bytes": len(gathered),
        "msm_reps": args.msm_reps,
    }
    if cpu and cpu.get("value"):
        out["gpu_over_cpu"] = value / cpu["value"]
    if args.stats_json:
        with open(args.stats_json, "w") as f:
            json.dump(stats, f, indent=1)
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
