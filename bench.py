#!/usr/bin/env python3
"""bench.py -- BASELINE metric: Groth16 constraints/sec (BLS12-381), plus MSM G1 Mpoints/s at 2^26.

Workload (BASELINE.json configs[2]): "Synthetic 2^26-constraint R1CS full Groth16 prove, 1 x MI355X".
A step = one full Groth16 prove of that circuit as the metric defines it ("witness and
R1CS in host memory, SRS resident on device" -> "192 B proof in host memory"): the witness upload from
page-locked host memory (overlapped with the previous step's proof, mi_groth16_prove_batch), witness
map, 7 NTTs, QAP division, 4 G1 MSMs (H, L, A, B_G1) + 1 G2 MSM (B_G2), proof assembly.  The 192-byte
proofs of all ranks are gathered to rank 0 over RCCL inside the timed region (the MultiProof assembly
of api/seal.hpp:306-308).  After the timer, every timed proof is pairing-verified (the C2 self-check
policy, api/seal.hpp:310-313) and the line carries "verified".

Multi-GPU: one process per GPU; by default each rank proves its own partition every step (PoSt /
PoRep partitions are independent proofs -- SURVEY.md 8e), so per-GPU work is fixed: weak scaling.
--partitions P runs BASELINE config 5's shape instead: every step proves P partitions round-robin over
the ranks (10 over 8 GPUs: two rounds on ranks 0 and 1) and all-gathers the P x 192-byte multi-proof.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--log-rows 26] [--partitions P]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Launch: under torch.distributed.run (WORLD_SIZE set) each process is one rank, and WORLD_SIZE must equal
--gpus.  Without a launcher, --gpus N > 1 makes this process a parent that, before touching the GPU, starts
N rank processes of itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free MASTER_PORT),
forwards rank 0's JSON line and exits non-zero if any rank fails (spawn_ranks).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "crypto3-fil-proofs_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# VALU bound of the accumulation kernel: v_mad_i64_i32 issue.  One wave64 MAD occupies its SIMD
# for 4 cycles: 1024 SIMDs x 64 lanes / 4 x 2.4 GHz = 39.3e12 lane-MADs/s.  (The dependent-chain
# microbench crypto3-fil-proofs_amd/microbench/madrate.hip sustains only 30.9e12 = 5.1 cycles,
# because each chain waits on its own previous MAD; the accumulation kernel's ISA and its measured
# time imply the 4-cycle rate.)  One Fq multiplication over 13 balanced 30-bit limbs = 338 MADs
# (field.h) -> 116.3e9 Fq-mul/s of pure MAD issue; the remaining gap to it is the non-MAD
# instructions (column carries, the quotient-digit selects of the exact zero test).
MAD_RATE = 1024 * 64 / 4 * 2.4e9
FQ_MUL_MADS = 338
FQ_MUL_PER_MIXED_ADD = {"G1": 10, "G2": 28}
# The chip's spec VALU issue rate (MI355X_MICROARCH.md "Wave scheduling": a wave64 VALU instruction issues
# over 2 cycles, 32 lanes/cycle per SIMD): 1024 SIMDs x 32 x 2.4 GHz lane-instructions/s.  Reported next to
# the measured-rate peaks so that a fraction of a measured instruction rate is not read as "done".
SPEC_VALU_LANE_INSTR = 1024 * 32 * 2.4e9
# ISA VALU instructions per G1 mixed addition (microbench/maddloop.hip's register form over
# the 13 x 30-bit field, 3,081 v_mad_i64_i32 + 1,915 other)
G1_MADD_VALU_INSTR = 3081 + 1915  # madd-2008-s: 8M + 2S over Fq
TOXIC_SEED = 0x5EED


def workload_name(log_rows, partitions=0, world=1):
    cfg = {26: " (BASELINE config 3)", 27: " (BASELINE config 4 shape: 32 GiB PoRep-sized, d = 2^27)"}
    base = f"synthetic 2^{log_rows}-constraint R1CS full Groth16 prove"
    if partitions:
        return (f"{partitions}-partition batch of the {base} (BASELINE config 5 shape: partitions "
                f"round-robin over {world} GPU(s))")
    return base + cfg.get(log_rows, "")


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


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, fg, synth_mod, ctx):
    """The oracle (oracle/, a CPU restatement of the same prover, OpenMP) on bounded samples of the
    same workload family: 2^a- and 2^b-constraint synthetic circuits (params generated on the GPU and
    exported, witness in host memory -> proof).  The rate at the target size is extrapolated from the
    two samples' measured scaling exponent and labelled as such.  Threads: OMP_NUM_THREADS (the GPU
    box allots each GPU a 16-CPU share and sets it to 16), else every CPU this process may run on."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py

    lease = cpu_lease()
    threads = lease["threads"]
    oracle_py.set_threads(threads)
    samples = []
    for lr in sorted(int(x) for x in str(args.cpu_log_rows).split(",")):
        sc = synth_mod.SynthCircuit(lr, args.n_in, args.seed)
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
        log(0, f"cpu baseline: 2^{lr} rows in {dt:.1f} s")
        proof_gpu = fg.prove(ctx, pk, circ, zb, r, s)
        samples.append({"log_rows": lr, "constraints": sc.n, "seconds": dt, "constraints_per_s": sc.n / dt,
                        "gpu_proof_bytes_identical": proof_cpu == proof_gpu})
        del op, oc, q, pk, circ, sc
    big = samples[-1]
    out = {
        "value": big["constraints_per_s"],
        "unit": "constraints/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle prove of the 2^{big['log_rows']}-row synthetic circuit ({big['constraints']} constraints), "
                  f"{big['seconds']:.2f} s with {threads} OpenMP threads on {cpu_model()}; GPU proof bytes identical: "
                  f"{all(x['gpu_proof_bytes_identical'] for x in samples)}",
        "cpu_model": cpu_model(),
        "host_cpus": os.cpu_count(),
        "lease": lease,
        "samples": samples,
    }
    if len(samples) >= 3:
        # least-squares fit of log t = alpha log n + c over every sample (>= 3 points), evaluated at the target
        xs = [math.log(x["constraints"]) for x in samples]
        ys = [math.log(x["seconds"]) for x in samples]
        mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
        alpha = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
        c0 = my - alpha * mx
        resid = max(abs(y - (alpha * x + c0)) for x, y in zip(xs, ys))
        n_t = (1 << args.log_rows) - args.n_in
        t_t = math.exp(alpha * math.log(n_t) + c0)
        out["extrapolated"] = {
            "label": "extrapolated",
            "log_rows": args.log_rows,
            "constraints": n_t,
            "seconds": t_t,
            "constraints_per_s": n_t / t_t,
            "model": f"least-squares log t = alpha log n + c over the {len(samples)} samples 2^"
                     f"{'/2^'.join(str(x['log_rows']) for x in samples)}, alpha = {alpha:.3f}, max |log residual| "
                     f"{resid:.3f}, {threads} threads",
        }
    return out


def cpu_lease():
    """The CPUs this process may really use, side by side: the affinity mask, the cgroup v2 cpu.max quota
    (quota / period CPUs, if any), and OMP_NUM_THREADS (the pool sets it to the lease's per-GPU share).
    threads = the quota when one is set, else OMP_NUM_THREADS, else the affinity mask; never more than the
    affinity mask."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    if quota:
        threads, basis = max(1, int(quota)), "cgroup cpu.max quota"
    elif omp:
        threads, basis = omp, "OMP_NUM_THREADS (the pool's per-GPU CPU share)"
    else:
        threads, basis = affinity, "affinity mask"
    threads = min(threads, affinity)
    return {"threads": threads, "basis": basis, "affinity_cpus": affinity, "cgroup_cpu_max_cpus": quota,
            "omp_num_threads": omp, "host_cpus": os.cpu_count()}


def tree_c_leg(args, fg, ctx, device, world):
    """tree C of one sub-tree (device-resident labels): column hashes + arity-8 tree, with its VALU
    roofline (v_mad_u64_u32 issue over the MADs of every Poseidon it runs) and the oracle's CPU rate."""
    import numpy as np
    import torch

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from tree_bench import MAD_RATE as TREE_MAD_RATE, mads_per_hash

    n, L = 1 << args.tree_log_nodes, 11
    g = torch.Generator(device=device)
    g.manual_seed(3)
    labels = torch.randint(0, 2 ** 62, (L * n, 4), dtype=torch.int64, device=device, generator=g)
    labels[:, 3] &= 0x0FFFFFFFFFFFFFFF  # < 2^252: canonical Fr
    base = torch.empty((n, 4), dtype=torch.int64, device=device)
    tree = torch.empty((fg.tree.get_merkle_tree_cache_size(n, 8, 0), 4), dtype=torch.int64, device=device)
    b = fg.tree.ColumnTreeBuilder(ctx, L, 8)
    b.add_final_columns_dev(labels.data_ptr(), n, base.data_ptr(), tree.data_ptr())
    ctx.synchronize()
    ctx.reset_stats()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        b.add_final_columns_dev(labels.data_ptr(), n, base.data_ptr(), tree.data_ptr())
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / reps
    st = ctx.stats()["poseidon"]
    node_hashes = (n - 1) // 7  # arity-8 tree over n leaves
    mads = n * mads_per_hash(11) + node_hashes * mads_per_hash(8)
    kern_s = st["ms"] * 1e-3 / reps
    out = {"workload": f"tree C of one sub-tree: 2^{args.tree_log_nodes} columns x 11 layers -> Poseidon-11 "
                       f"column hashes -> arity-8 Poseidon tree (device-resident labels)",
           "columns_per_s": n / dt, "ms_per_tree": dt * 1e3, "kernel_ms_per_tree": kern_s * 1e3,
           "valu_roofline": {"kernel": "k_poseidon<12> + k_poseidon<9>", "bound": "valu (v_mad_i64_i32 issue)",
                             "mads_per_tree": mads, "achieved_mads_per_s": mads / kern_s,
                             "peak_mads_per_s": TREE_MAD_RATE, "frac": mads / kern_s / TREE_MAD_RATE,
                             "spec_issue": {"peak_lane_instr_per_s": SPEC_VALU_LANE_INSTR,
                                            "frac_mads_only": mads / kern_s / SPEC_VALU_LANE_INSTR,
                                            "note": "v_mad_u64_u32 lane-instructions alone against the spec "
                                                    "VALU issue rate (a lower bound on issue use: the other "
                                                    "VALU instructions are not counted)"}},
           "hbm_algorithmic_GBps": (n * (32 * L + 32) + node_hashes * 9 * 32) / kern_s / 1e9}
    if world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_py

        threads = cpu_lease()["threads"]
        oracle_py.set_threads(threads)
        m = 4096
        sample = labels.view(L, n, 4)[:, :m].permute(1, 0, 2).contiguous().cpu().numpy().view(np.uint8).tobytes()
        t0 = time.perf_counter()
        oracle_py.poseidon_hash_sparse(11, sample)
        dtc = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": m / dtc, "unit": "column hashes/s", "cores": threads, "kind": "port",
                               "sample": f"{m} Poseidon-11 column hashes of the same labels by the oracle in the "
                                         f"optimised (sparse-round) form Filecoin's CPU hasher uses, 64-bit-limb "
                                         f"Montgomery, OpenMP, on {cpu_model()}"}
        out["gpu_over_cpu"] = out["columns_per_s"] / out["cpu_baseline"]["value"]
    del labels, base, tree
    return out


# SHA-256 compression cost model for the SDR label kernel (VALU lane-ops, gfx950 3-input forms): per round
# Sigma0/Sigma1 3 v_alignbit + 1 v_bitop3 (xor3) each, Ch and Maj 1 v_bitop3 each, T1 2 v_add3, e 1 add,
# a 1 v_add3 = 14; per schedule word sigma0/sigma1 2 v_alignbit + 1 shift + 1 xor3 each, v_add3 + add = 10;
# 8 feed-forward adds.  The compiled block loop issues 1,410 VALU per compression (this + the byte swaps).
SHA256_OPS_PER_COMPRESSION = 64 * 14 + 48 * 10 + 8
# Peak: the measured chip-wide issue rates of the model's instructions (crypto3-fil-proofs_amd/microbench/
# intrate.hip, profiles/r02_intrate_microbench.jsonl): v_alignbit_b32 and v_add3_u32 3.54e13 lane-ops/s,
# v_bitop3_b32 / v_add_u32 / shifts 5.31e13.  Per compression the model holds 816 of the former (6 + 4
# rotations per round / schedule word, 3 + 1 add3) and 568 of the latter.
SHA256_SLOW_OPS, SHA256_FAST_OPS = 64 * 6 + 48 * 4 + 64 * 3 + 48, 64 * 14 + 48 * 10 + 8 - (64 * 9 + 48 * 5)
SHA256_PEAK_COMPRESSIONS = 1.0 / (SHA256_SLOW_OPS / 3.54e13 + SHA256_FAST_OPS / 5.31e13)
VALU_LANE_OPS = SHA256_PEAK_COMPRESSIONS * SHA256_OPS_PER_COMPRESSION  # model lane-ops/s at that peak


def sdr_leg(args, fg, ctx, device, world):
    """labelling-proof labels of 2^N challenges gathered from 11 device-resident layers of 2^20
    nodes (6 base + 8 expander parents each, repeated to 37: 20 SHA-256 compressions per label), with the
    VALU roofline of k_sdr_labels_gather and the oracle's CPU rate on a sample."""
    import numpy as np
    import torch

    n_layers, nodes, count = 11, 1 << 20, 1 << args.sdr_log_labels
    g = torch.Generator(device=device)
    g.manual_seed(21)
    labels = torch.randint(0, 256, (n_layers * nodes * 32,), dtype=torch.uint8, device=device, generator=g)
    layers = torch.randint(1, n_layers + 1, (count,), dtype=torch.int32, device=device, generator=g)
    chal = torch.randint(1, nodes, (count,), dtype=torch.int64, device=device, generator=g)
    pidx = torch.randint(0, nodes, (count * 14,), dtype=torch.int32, device=device, generator=g)
    out = torch.empty(count * 32, dtype=torch.uint8, device=device)
    rid = bytes(range(32))
    torch.cuda.synchronize()

    def run():
        fg.sdr.labeling_proofs_dev(ctx, rid, n_layers, nodes, labels.data_ptr(), count, layers.data_ptr(),
                                   chal.data_ptr(), pidx.data_ptr(), out.data_ptr())

    run()
    ctx.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / reps
    compressions = count * 20
    ops = compressions * SHA256_OPS_PER_COMPRESSION
    res = {"workload": f"SDR labelling-proof labels: 2^{args.sdr_log_labels} challenges x 37 parents (6 base + 8 "
                       f"expander, repeated) gathered from 11 device-resident layers of 2^20 nodes; SHA-256 over "
                       f"1248 B each",
           "labels_per_s": count / dt, "ms_per_batch": dt * 1e3,
           "note": "wall time per call includes the device-side index range check (k_sdr_check) and one host "
                   "synchronisation; rocprofv3 gives the kernel alone",
           "valu_roofline": {"kernel": "k_sdr_labels_gather", "bound": "valu (32-bit integer issue)",
                             "ops_per_compression": SHA256_OPS_PER_COMPRESSION, "compressions_per_label": 20,
                             "achieved_ops_per_s": ops / dt, "peak_ops_per_s": VALU_LANE_OPS,
                             "peak_source": "measured issue rates of the model's instructions "
                                            "(microbench/intrate.hip, profiles/r02_intrate_microbench.jsonl)",
                             "frac": ops / dt / VALU_LANE_OPS,
                             "spec_issue": {"peak_lane_instr_per_s": SPEC_VALU_LANE_INSTR,
                                            "frac": ops / dt / SPEC_VALU_LANE_INSTR,
                                            "note": "the model's lane-ops against the spec VALU issue rate "
                                                    "(32 lanes/cycle/SIMD, 2.4 GHz)"}},
           "hbm_algorithmic_GBps": count * (14 * 32 + 4 + 8 + 56 + 32) / dt / 1e9,
           "traffic_source": "profiles/r02_sdr_summary.json (FETCH_SIZE 2,644 B per label raw vs 548 B "
                             "algorithmic: line-granular random 32-B parent gathers; WRITE_SIZE 32 B per label)"}
    if world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_py

        threads = cpu_lease()["threads"]
        oracle_py.set_threads(threads)
        m = 1 << 19
        par = np.random.default_rng(1).integers(0, 256, 32 * 14 * m, dtype=np.uint8).tobytes()
        lay = np.random.default_rng(2).integers(2, 12, m, dtype=np.uint32)
        nod = np.random.default_rng(3).integers(1, 1 << 20, m, dtype=np.uint64)
        t0 = time.perf_counter()
        oracle_py.sdr_labels(rid, lay, nod, par, 14)
        dtc = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": m / dtc, "unit": "labels/s", "cores": threads, "kind": "port",
                               "sample": f"{m} labels (14 parents repeated to 37) by the oracle's scalar C SHA-256, "
                                         f"OpenMP, on {cpu_model()}"}
        res["gpu_over_cpu"] = res["labels_per_s"] / res["cpu_baseline"]["value"]
    del labels, layers, chal, pidx, out
    return res


def uniform_leg(args, fg, synth_mod, ctx):
    """The headline shape with a uniform witness: the generator's boolean rows become packing
    rows (MI_SYNTH_UNIFORM_WITNESS), so every MSM scalar is a uniform field element and L / A / B issue ~12 mixed
    additions per point instead of the headline witness's ~8.4.  Same domain, same row shapes, host (pinned)
    witness; one warm-up, `uniform_steps` timed proofs in one batch, every proof pairing-verified."""
    import gc

    import numpy as np

    t0 = time.perf_counter()
    sc = synth_mod.SynthCircuit(args.log_rows, args.n_in, args.seed, uniform=True)
    circ = sc.load(ctx)
    pk = fg.generate_random_parameters(ctx, circ, splitmix_frs(TOXIC_SEED, 5))
    ctx.synchronize()
    t_setup = time.perf_counter() - t0
    z = fg.HostBuffer(32 * sc.num_vars)
    np.copyto(z.array, sc.z_array())
    k = args.uniform_steps
    blind = splitmix_frs(7000, 2 * (k + 1))
    fg.prove_batch(ctx, pk, circ, [z], [(blind[0], blind[1])])
    ctx.synchronize()
    ctx.reset_stats()
    t1 = time.perf_counter()
    proofs = fg.prove_batch(ctx, pk, circ, [z] * k, [(blind[2 * i + 2], blind[2 * i + 3]) for i in range(k)])
    ctx.synchronize()
    dt = (time.perf_counter() - t1) / k
    st = ctx.stats()
    vk, ic = pk.verifying_key()
    pub = z.array[32:32 * sc.n_in].tobytes()
    verified = bool(fg.verify_batch(vk, ic, [pub] * len(proofs), proofs))
    acc = st["accum_g1"]
    out = {"workload": f"{workload_name(args.log_rows)} with a uniform witness (no boolean rows: every aux value a "
                       f"uniform field element or a product of such)",
           "value": sc.n / dt, "unit": "constraints/s", "ms_per_proof": dt * 1e3, "proofs": k, "verified": verified,
           "g1_mixed_adds_per_launch": acc["madds"] / max(acc["launches"], 1),
           "accum_g1_ms_per_launch": acc["ms"] / max(acc["launches"], 1), "setup_s": t_setup,
           "a_query": circ.n_a, "b_query": circ.n_b}
    del proofs, z, pk, circ, sc
    gc.collect()
    return out


def config4_leg(args, fg, synth_mod, ctx):
    """BASELINE config 4 (the north-star target: a 32 GiB Seal-PoRep-sized circuit, ~1.3e8 constraints,
    d = 2^27) on the same GPU after the config-3 objects are freed: host (pinned) witness, one warm-up and
    `config4_steps` timed proofs with overlapped uploads, every proof pairing-verified."""
    import gc

    import numpy as np

    lr = args.config4_log_rows
    t0 = time.perf_counter()
    sc = synth_mod.SynthCircuit(lr, args.n_in, args.seed)
    circ = sc.load(ctx)
    pk = fg.generate_random_parameters(ctx, circ, splitmix_frs(TOXIC_SEED, 5))
    ctx.synchronize()
    t_setup = time.perf_counter() - t0
    log(0, f"config 4 setup {t_setup:.1f} s")
    z = fg.HostBuffer(32 * sc.num_vars)
    np.copyto(z.array, sc.z_array())
    blind = splitmix_frs(4000, 2 * (1 + args.config4_steps))
    fg.prove_batch(ctx, pk, circ, [z], [(blind[0], blind[1])])
    ctx.synchronize()
    t1 = time.perf_counter()
    proofs = fg.prove_batch(ctx, pk, circ, [z] * args.config4_steps,
                            [(blind[2 * k + 2], blind[2 * k + 3]) for k in range(args.config4_steps)])
    ctx.synchronize()
    dt = (time.perf_counter() - t1) / args.config4_steps
    vk, ic = pk.verifying_key()
    pub = z.array[32:32 * sc.n_in].tobytes()
    verified = bool(fg.verify_batch(vk, ic, [pub] * len(proofs), proofs))
    out = {"workload": f"BASELINE config 4 shape: synthetic 2^{lr}-domain R1CS ({sc.n} constraints, 32 GiB "
                       f"Seal-PoRep-sized), host (pinned) witness",
           "value": sc.n / dt, "unit": "constraints/s", "ms_per_proof": dt * 1e3, "proofs": len(proofs),
           "verified": verified, "setup_s": t_setup, "domain": circ.d, "a_query": circ.n_a, "b_query": circ.n_b}
    del proofs, z, pk, circ, sc
    gc.collect()
    return out


def stacked_leg(args, fg, ctx, device, world):
    """SURVEY 8(f)#3 + BASELINE config 4 on the real circuit: one 32 GiB stacked-PoRep partition (11 layers, 18
    challenges, 2^30 nodes, tree C / R-last 8-8; 130,278,541 constraints, domain 2^27).  The R1CS is built
    on the host (once per shape) and the proving key generated on the GPU (setup, untimed); then the
    partition's witness is generated on the GPU from its vanilla openings (a synthetic consistent
    instance: sparse trees, labels from the label kernel) and proven, every proof pairing-verified.  The
    witness kernels are HBM-bound by the 32-byte variables they write; the roofline is reported against
    8 TB/s.  CPU baseline: the oracle's Python synthesis (one thread) on the 2-layer reference shape."""
    import gc

    import numpy as np
    import torch

    from fil_groth16 import stacked

    t0 = time.perf_counter()
    sc_ = stacked.StackedCircuit(args.stacked_layers, args.stacked_challenges, 1 << args.stacked_log_nodes, 8, 8, 0)
    t_build = time.perf_counter() - t0
    inst = stacked.synthetic_instance(ctx, sc_, seed=32)
    slots = stacked.slots_of(sc_, inst)
    t_inst = time.perf_counter() - t0 - t_build
    circ = sc_.load(ctx)
    pk = fg.generate_random_parameters(ctx, circ, splitmix_frs(TOXIC_SEED, 5))
    ctx.synchronize()
    t_setup = time.perf_counter() - t0
    log(0, f"stacked setup {t_setup:.1f} s")
    nv = sc_.num_vars
    sd = torch.from_numpy(np.frombuffer(slots, dtype=np.uint8).copy()).to(device)
    z = torch.empty(32 * nv, dtype=torch.uint8, device=device)
    torch.cuda.synchronize()
    sc_.witness_dev(ctx, sd.data_ptr(), z.data_ptr())  # warm (program upload)
    bad, _ = stacked.circuit_check_dev(ctx, circ, z.data_ptr())
    ctx.reset_stats()
    reps = args.stacked_reps
    tw = time.perf_counter()
    for _ in range(reps):
        sc_.witness_dev(ctx, sd.data_ptr(), z.data_ptr())
    ctx.synchronize()
    tw = (time.perf_counter() - tw) / reps
    st = ctx.stats()
    blind = splitmix_frs(5000, 2 * (reps + 1))
    fg.prove(ctx, pk, circ, z.data_ptr(), blind[0], blind[1])
    ctx.synchronize()
    tp = time.perf_counter()
    proofs = []
    for k in range(reps):
        sc_.witness_dev(ctx, sd.data_ptr(), z.data_ptr())
        proofs.append(fg.prove(ctx, pk, circ, z.data_ptr(), blind[2 * k + 2], blind[2 * k + 3]))
    ctx.synchronize()
    tp = (time.perf_counter() - tp) / reps
    vk, ic = pk.verifying_key()
    pub = sc_.public_inputs(slots)
    verified = bool(fg.verify_batch(vk, ic, [pub] * len(proofs), proofs))
    wbytes = 32 * nv
    res = {"workload": f"32 GiB stacked-PoRep partition: {args.stacked_layers} layers x {args.stacked_challenges} "
                       f"challenges, 2^{args.stacked_log_nodes} nodes, tree C / R-last 8-8 "
                       f"({sc_.num_constraints} constraints, {nv} variables, domain 2^{circ.d.bit_length() - 1}); "
                       f"synthetic consistent instance",
           "constraints": sc_.num_constraints, "variables": nv, "r1cs_entries": sc_.info["r1cs_entries"],
           "witness_ms": tw * 1e3, "witness_variables_per_s": nv / tw,
           "witness_phases_ms_per_partition": {k: st[k]["ms"] / reps for k in ("wit_a", "wit_sha", "wit_pos")},
           "witness_satisfies_r1cs": bad == 0,
           "witness_plus_prove_ms": tp * 1e3, "constraints_per_s": sc_.num_constraints / tp,
           "proofs": len(proofs), "verified": verified,
           "witness_roofline": {"bound": "hbm", "achieved": wbytes / tw / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": wbytes / tw / 1e9 / HBM_PEAK_GBS,
                                "algorithmic_bytes": wbytes, "note": "32 B written per variable; reads are the "
                                "instance slots and operand variables (small)"},
           "setup_s": {"r1cs_build": t_build, "instance": t_inst, "load_and_keygen": t_setup - t_build - t_inst}}
    if world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import stacked_circuit as osc
        import stacked_instance as osi

        oinst = osi.generate(8, 2, (8, 0, 0), 1, seed=3)
        t1 = time.perf_counter()
        ocs = osc.CS(with_constraints=False)
        osc.stacked_circuit(ocs, oinst, 2, 8, (8, 0, 0))
        dtc = time.perf_counter() - t1
        nvo = len(ocs.inputs) + len(ocs.aux)
        res["cpu_baseline"] = {"value": nvo / dtc, "unit": "witness variables/s", "cores": 1, "kind": "port",
                               "sample": f"oracle/stacked_circuit.py (Python, one thread) synthesising the reference "
                                         f"test shape (2 layers, 1 challenge, 8 nodes: {nvo} variables) in "
                                         f"{dtc:.1f} s on {cpu_model()}"}
        res["gpu_over_cpu_witness"] = res["witness_variables_per_s"] / res["cpu_baseline"]["value"]
    del pk, circ, z, sd, sc_
    gc.collect()
    torch.cuda.synchronize()
    return res


def params_roundtrip(fg, ctx, circ, pk, zhost, rs):
    """setup_s.params_load: the resident key written as a bellman/filecoin v28 params file under TMPDIR, loaded back
    through mi_params_load unchecked (mmap + decode + upload) and checked (+ every point's subgroup test), and a proof
    from the checked key compared byte for byte with the resident key's.  The file normally stays in the page cache
    after the write, so the rates are the load path's, not a cold disk's (disk rate unmeasured)."""
    import gc
    import shutil
    import tempfile

    nbytes = 96 * (pk.n_h + pk.n_l + pk.n_a + pk.n_b) + 192 * pk.n_b + 96 * (circ.num_inputs + 9)
    tmpd = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    rec = {"file_bytes": nbytes, "disk_free_bytes": shutil.disk_usage(tmpd).free,
           "note": "page-cache rates (the file was just written); cold-disk rate unmeasured"}
    try:
        if rec["disk_free_bytes"] < 1.1 * nbytes:
            rec["skipped"] = "scratch disk too small for the params file"
            return rec
        path = os.path.join(tmpd, "key.params")
        t0 = time.perf_counter()
        pk.write_params(path)
        rec["write_s"] = time.perf_counter() - t0
        want = fg.prove_batch(ctx, pk, circ, [zhost], [rs])[0]
        for checked in (False, True):
            t0 = time.perf_counter()
            pk2 = fg.ProvingKey.load_params(ctx, circ, path, checked=checked)
            ctx.synchronize()
            t = time.perf_counter() - t0
            key = "load_checked" if checked else "load"
            rec[key + "_s"] = t
            rec[key + "_GBps"] = nbytes / t / 1e9
            if checked:
                rec["proof_equal"] = fg.prove_batch(ctx, pk2, circ, [zhost], [rs])[0] == want
            del pk2
            gc.collect()
        rec["subgroup_check_s"] = rec["load_checked_s"] - rec["load_s"]
    finally:
        shutil.rmtree(tmpd, ignore_errors=True)
    return rec


def window_post_leg(args, fg, ctx, device, rank, world, gdev, dist):
    """The Window-PoSt circuit itself: partitions of --post-sectors 32 GiB sectors x
    --post-challenges challenges (2349 x 10 = 125,279,217 constraints, constants.hpp:85-89; domain 2^27).
    Setup (untimed): the R1CS built on the host and uploaded in compact form, the proving key generated on the
    GPU from the fixed toxic waste (the same SRS on every rank), one synthetic partition instance per
    partition (sparse trees R-last, challenges by generate_leaf_challenge) resident in HBM.  Timed: per
    partition the GPU witness (mi_stacked_witness_dev) and the proof.
      world == 1: --post-reps partitions back to back on one GPU (the per-partition rate of config 5).
      world > 1 : BASELINE config 5 -- --post-partitions (10) partitions over the ranks: P - P % W round-robin as
                  whole proofs, the P % W tail partitions each over a group of ranks in latency mode (at 8 GPUs:
                  partitions 0-7 whole, 8 and 9 over four GPUs each; MI_C5_SCHEDULE=roundrobin leaves them
                  to a second round on ranks 0 and 1); the P x 192-byte multi-proof (whole proofs + shares)
                  all-gathered over RCCL, the makespan max over ranks; rank 0 pairing-verifies every gathered
                  proof against each partition's inputs."""
    import gc

    import numpy as np
    import torch

    from fil_groth16 import stacked
    from fil_groth16.compound import shard_partitions
    from fil_groth16.distributed import (agree_float, balanced_schedule, calibrate_hsplit, calibrate_lead_share,
                                         hsplit_fractions, hsplit_shares, latency_ranges, latency_ranges_hsplit,
                                         lead_share_from_times, prove_partitions, prove_partitions_balanced,
                                         destroy_group_broadcasters, group_broadcaster)

    S, C, nodes = args.post_sectors, args.post_challenges, 1 << args.post_log_nodes
    try:
        avail_gb = int(next(l for l in open("/proc/meminfo") if l.startswith("MemAvailable")).split()[1]) / 1e6
    except (OSError, StopIteration):
        avail_gb = None
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    need_gb = 25.0 * S / 2349  # compact R1CS build peak + instances, per rank
    if avail_gb is not None and avail_gb < local_world * need_gb:
        return {"skipped": f"MemAvailable {avail_gb:.0f} GB < {local_world} ranks x {need_gb:.0f} GB"}
    t0 = time.perf_counter()
    pc = stacked.FallbackPoStCircuit(S, C, nodes, 8, 8, 0)
    t_build = time.perf_counter() - t0
    circ = pc.load(ctx)
    pk = fg.generate_random_parameters(ctx, circ, splitmix_frs(TOXIC_SEED, 5))
    P = args.post_partitions if world > 1 else args.post_reps
    # config 5's schedule: "balanced" (default) proves the P % W tail partitions in latency mode over rank
    # groups (distributed.balanced_schedule); "roundrobin" leaves them to a last round on P % W ranks
    schedule = os.environ.get("MI_C5_SCHEDULE", "balanced") if world > 1 else "local"
    whole, tail = balanced_schedule(P, world) if schedule == "balanced" else \
        ([shard_partitions(P, r, world) for r in range(world)], [])
    if world == 1:
        whole = [list(range(P))]
    mine = whole[rank] + [p for p, rs in tail if rank in rs]
    slots, sdev = {}, {}
    for p in mine:  # each rank makes only its own partitions' instances (~12 s each for 2349 sectors)
        _, sectors = stacked.synthetic_post_instance(ctx, pc, seed=4000 + p, partition=p)
        slots[p] = stacked.post_slots(pc, sectors)
        sdev[p] = torch.from_numpy(np.frombuffer(slots[p], dtype=np.uint8).copy()).to(device)
    # rank 0 verifies every partition: the public inputs travel to it (one all-gather of fixed-size records:
    # partition id + 32 x (inputs - 1) bytes, at most max(|mine|) per rank) instead of rank 0 building every
    # instance itself
    pub_len = 32 * (pc.num_inputs - 1)
    pubs_of = {p: pc.public_inputs(slots[p]) for p in mine}
    if dist:
        kmax = max(len(whole[r]) + sum(1 for _, rs in tail if r in rs) for r in range(world))
        rec = np.zeros((kmax, 8 + pub_len), dtype=np.uint8)
        rec[:, :8] = 0xFF
        for i, p in enumerate(mine):
            rec[i, :8] = np.frombuffer(int(p).to_bytes(8, "little"), dtype=np.uint8)
            rec[i, 8:] = np.frombuffer(pubs_of[p], dtype=np.uint8)
        t = torch.from_numpy(rec).to(gdev)
        bufs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(bufs, t)
        if rank == 0:
            for b in bufs:
                for row in b.cpu().numpy():
                    p = int.from_bytes(row[:8].tobytes(), "little")
                    if p < P:
                        pubs_of.setdefault(p, row[8:].tobytes())
        del t, bufs
    z = torch.empty(32 * pc.num_vars, dtype=torch.uint8, device=device)
    ctx.synchronize()
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t0
    log(rank, f"Window-PoSt setup {t_setup:.1f} s (R1CS {t_build:.1f} s, key, {len(slots)} partition instances on "
              f"rank 0)")
    blind = splitmix_frs(9000 + rank, 2 * (len(mine) * (args.config5_steps + 1) + 2))
    state = {"k": 2}

    def prove_ids(ids):
        out = []
        for p in ids:
            pc.witness_dev(ctx, sdev[p].data_ptr(), z.data_ptr())
            k = state["k"]
            state["k"] += 2
            out.append(fg.prove(ctx, pk, circ, z.data_ptr(), blind[k], blind[k + 1]))
        return out

    vk, ic = pk.verifying_key()

    # latency-mode groups compute H once and split it (MI_C5_LATENCY=h_split, default): the group's
    # lead rank runs the witness map and the NTT chain (mi_groth16_h_coeffs_dev), broadcasts the d H coefficients
    # over the group (RCCL, asynchronous) and takes a calibrated slice of H; the others prove their L / A / B
    # slices first, then their H slices from the broadcast (distributed.hsplit_shares).  MI_C5_LATENCY=h_once: the
    # lead keeps the whole H MSM (round 4); slices: every rank repeats H and takes equal slices.
    latency = os.environ.get("MI_C5_LATENCY", "h_split")
    sizes = (pk.n_h, pk.n_l, pk.n_a, pk.n_b)
    calib = {}
    hbuf = torch.zeros(32 * circ.d, dtype=torch.uint8, device=device) if latency == "h_split" else None

    def share_fn(p, k, g, bcast=None):
        pc.witness_dev(ctx, sdev[p].data_ptr(), z.data_ptr())
        if latency == "slices":
            return fg.prove_share(ctx, pk, circ, z.data_ptr(), k, g)
        if latency == "h_once":
            rg = latency_ranges(sizes, g, lead_share_from_times(calib["t_h_ms"], calib["t_lab_ms"], g))
            return fg.prove_share_ranges(ctx, pk, circ, z.data_ptr(), rg[k])
        rg = latency_ranges_hsplit(sizes, g, *hsplit_fractions(calib["t_qap_ms"], calib["t_hmsm_ms"],
                                                               calib["t_lab_ms"], g))

        def h_coeffs(*arg):
            if not arg:  # the lead: witness map + NTT chain into hbuf
                fg.h_coeffs_dev(ctx, circ, z.data_ptr(), hbuf.data_ptr())
            return hbuf

        def one(ranges, h):
            return fg.prove_share_ranges(ctx, pk, circ, z.data_ptr(), ranges,
                                         h_dev=h.data_ptr() if h is not None else None)

        return hsplit_shares(k, rg, h_coeffs, one, bcast or (lambda t: (lambda: t)))

    def assemble_fn(p, shares):  # the same blinding on every rank of the group
        return fg.assemble(vk, shares, *splitmix_frs(9500 + p, 2))

    if latency != "slices" and (tail or (world == 1 and args.post_share_groups)):
        # one GPU's times of the parts of a proof (h_once: H part; L, A, B part -- h_split: NTT chain; H MSM; L, A,
        # B), rank 0's agreed by every rank
        keys = ("t_qap_ms", "t_hmsm_ms", "t_lab_ms") if latency == "h_split" else ("t_h_ms", "t_lab_ms")
        if mine:
            pc.witness_dev(ctx, sdev[mine[0]].data_ptr(), z.data_ptr())
            if latency == "h_split":
                t = calibrate_hsplit(ctx, pk, circ, z.data_ptr(), hbuf.data_ptr())
            else:
                _, t = calibrate_lead_share(ctx, pk, circ, z.data_ptr(), 2)
        else:
            t = {k: 0.0 for k in keys}
        calib = {k: agree_float(t[k], rank, gdev) if dist else t[k] for k in keys}
    if mine:  # warm-up (program upload, plans)
        pc.witness_dev(ctx, sdev[mine[0]].data_ptr(), z.data_ptr())
        if whole[rank]:
            fg.prove(ctx, pk, circ, z.data_ptr(), blind[0], blind[1])
        for p, rs in tail:
            if rank in rs:
                share_fn(p, rs.index(rank), len(rs))
    if dist and tail and latency == "h_split":
        for p, rs in tail:  # every rank, in schedule order: the tail groups and their first broadcast, untimed
            group_broadcaster(rs, gdev)
    ctx.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.reset_stats()
    steps = args.config5_steps if world > 1 else 1
    t1 = time.perf_counter()
    multi = []
    for _ in range(steps):
        if world > 1:
            multi.append(prove_partitions_balanced(prove_ids, share_fn, assemble_fn, P, rank, world, gdev,
                                                   group_bcast=latency == "h_split")
                         if tail else prove_partitions(prove_ids, P, rank, world, gdev))
        else:
            multi.append(b"".join(prove_ids(mine)))
    ctx.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t1
    mine_dt = dt
    st = ctx.stats()
    if world > 1 and tail and latency == "h_split":
        destroy_group_broadcasters()  # the tail groups' communicators (created once, at the warm-up step)
    # one GPU: the latency-mode shares the balanced config-5 schedule gives a tail partition, timed one after
    # another (slowest share = that group's tail on g GPUs), assembled and compared with the whole proof
    shares_res = None
    if world == 1 and args.post_share_groups and mine:
        p0 = mine[0]
        rs0 = splitmix_frs(9500 + p0, 2)
        pc.witness_dev(ctx, sdev[p0].data_ptr(), z.data_ptr())
        ref = fg.prove(ctx, pk, circ, z.data_ptr(), *rs0)
        shares_res = {}
        for g in [int(x) for x in args.post_share_groups.split(",") if x]:
            share_fn(p0, 0, g)  # warm (slice plans)
            ctx.synchronize()
            ts, shs = [], []
            for k in range(g):  # rank k's shares in turn (h_split: rank 0's H coefficients stay in hbuf)
                t2 = time.perf_counter()
                got = share_fn(p0, k, g)
                ctx.synchronize()
                ts.append(time.perf_counter() - t2)
                shs += [got] if isinstance(got, (bytes, bytearray)) else list(got)
            mean = sum(ts) / len(ts)
            shares_res[str(g)] = {"share_ms": [1e3 * x for x in ts], "slowest_ms": 1e3 * max(ts),
                                  "mean_ms": 1e3 * mean, "slowest_over_mean": max(ts) / mean,
                                  "assembled_equals_whole_proof": fg.assemble(vk, shs, *rs0) == ref,
                                  "mode": latency}
            if latency == "h_once":
                shares_res[str(g)]["lead_share"] = lead_share_from_times(calib["t_h_ms"], calib["t_lab_ms"], g)
            elif latency == "h_split":
                hl, fl = hsplit_fractions(calib["t_qap_ms"], calib["t_hmsm_ms"], calib["t_lab_ms"], g)
                # the lead's broadcast of d x 32 B runs beside its own share (asynchronous); the others need H only
                # after their L / A / B slices: estimated at one xGMI link (~64 GB/s effective), a projection
                bc_ms = 32 * circ.d / 64e9 * 1e3
                shares_res[str(g)].update(h_lead=hl, lab_lead=fl, h_bcast_ms_estimate=bc_ms,
                                          h_needed_after_ms=1e3 * min(ts[1:]) if g > 1 else None)
    if dist:
        tt = torch.tensor([dt], dtype=torch.float64, device=gdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    out = None
    if rank == 0:
        proofs = [m[192 * i:192 * (i + 1)] for m in multi for i in range(P)]
        pubs = [pubs_of[i] for _ in multi for i in range(P)]
        verified = bool(fg.verify_batch(vk, ic, pubs, proofs))
        per_step = dt / steps
        n = pc.num_constraints
        out = {"workload": f"Window-PoSt partitions of the real circuit: {S} sectors x {C} challenges over 2^"
                           f"{args.post_log_nodes}-node 8-8-0 trees R-last ({n} constraints, {pc.num_inputs} inputs, "
                           f"domain 2^{circ.d.bit_length() - 1}); synthetic consistent partitions; timed = GPU "
                           f"witness + proof per partition" +
                           (f"; BASELINE config 5: {P} partitions over {world} GPUs ({schedule} schedule), {P} x 192-byte "
                            f"multi-proof all-gathered" if world > 1 else f"; {P} partitions on one GPU"),
               "partitions": P, "n_gpus": world, "constraints": n, "steps": steps,
               "makespan_s": per_step, "proofs_per_s": P / per_step, "constraints_per_s": P * n / per_step,
               "ms_per_partition_rank0": 1e3 * mine_dt / steps / max(1, len(mine)),
               "witness_ms_per_partition_rank0": (st["wit_a"]["ms"] + st["wit_sha"]["ms"] + st["wit_pos"]["ms"]) /
                                                 max(1, steps * len(mine)),
               "verified": verified, "verified_proofs": len(proofs),
               "setup_s": {"r1cs_build": t_build, "total": t_setup}, "host_mem_available_gb": avail_gb}
        if shares_res:
            tp1 = 1e3 * mine_dt / steps / max(1, len(mine))
            out["latency_mode_shares"] = shares_res
            if calib:
                out["latency_mode_calibration_ms"] = calib
            out["config5_projection"] = {
                "note": "projected from this GPU's times (witness + share per rank, ranks independent): 10 "
                        "partitions; balanced = P - P % W whole partitions round-robin, then each of the P % W "
                        "tail partitions over W / (P % W) GPUs in latency mode (" + latency + ": " +
                        {"h_split": "the group's lead rank alone computes H and broadcasts it, every rank proves a "
                                    "slice of H, L, A and B",
                         "h_once": "the group's lead rank alone computes H and proves the whole H MSM"}.get(
                            latency, "every rank repeats H, equal slices") + "); a PROJECTION, not a measurement",
                "w8_roundrobin_makespan_ms": 2 * tp1,
                "w8_balanced_makespan_ms": tp1 + shares_res["4"]["slowest_ms"] if "4" in shares_res else None,
                "w4_roundrobin_makespan_ms": 3 * tp1,
                "w4_balanced_makespan_ms": 2 * tp1 + shares_res["2"]["slowest_ms"] if "2" in shares_res else None}
        if world > 1:
            out["schedule"] = schedule
            out["latency_mode"] = latency if tail else None
            if calib:
                out["latency_mode_calibration_ms"] = calib
            out["per_rank_partitions"] = [len(w) for w in whole]
            out["split_partitions"] = [{"partition": p, "ranks": rs} for p, rs in tail]
    del pk, circ, z, sdev, pc
    gc.collect()
    torch.cuda.synchronize()
    return out


def spawn_ranks(n, argv):
    """`bench.py --gpus N` with no launcher: N child ranks of this script, one per GPU (LOCAL_RANK = rank),
    rendezvous on 127.0.0.1.  This process never touches the GPU (no torch import), so starting children is
    safe.  Rank 0's stdout (the JSON line) is forwarded; every rank's stderr passes through.  If any rank exits
    non-zero the others are stopped (they would wait in a collective) and the parent exits with that code."""
    import socket
    import subprocess
    import threading

    port = os.environ.get("MASTER_PORT")
    if not port:
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = str(sk.getsockname()[1])
    procs, lines = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr))
    import signal

    def stop(signum, _frame):  # a time limit on the parent ends the ranks too
        for p in procs:
            if p.poll() is None:
                p.kill()
        sys.exit(128 + signum)

    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    reader = threading.Thread(target=lambda: lines.extend(procs[0].stdout), daemon=True)
    reader.start()
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0]
            print(f"[bench] a rank exited with {rc}; stopping the others", file=sys.stderr, flush=True)
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(0.2)
    reader.join(timeout=10)
    for ln in lines:
        sys.stdout.write(ln.decode() if isinstance(ln, bytes) else ln)
    sys.stdout.flush()
    return rc


def winning_post_leg(args, fg, ctx, device):
    """SURVEY 8(a) a2 generate_winning_post (api/post.hpp:178-230) on the real circuit at the reference's shape:
    winning_post_setup_params (parameters.hpp:58-68) turns 66 challenges over 1 sector into 66 circuit sectors x
    1 challenge over the one replica (2^30-node 8-8-0 tree R-last at 32 GiB: 370,590 constraints, 133 inputs,
    domain 2^19).  Winning PoSt is the latency-critical single-GPU path (SURVEY CS-3): timed = GPU witness +
    proof of one partition, --winning-reps times back to back (latency per proof, not throughput), every proof
    pairing-verified after the timer."""
    import gc

    import numpy as np
    import torch

    from fil_groth16 import stacked

    t0 = time.perf_counter()
    wc = stacked.WinningPoStCircuit(1 << args.winning_log_nodes, 8, 8, 0)
    t_build = time.perf_counter() - t0
    _, sectors = stacked.synthetic_winning_post_instance(ctx, wc, seed=66)
    slots = stacked.post_slots(wc, sectors)
    circ = wc.load(ctx)
    pk = fg.generate_random_parameters(ctx, circ, splitmix_frs(TOXIC_SEED, 5))
    sd = torch.from_numpy(np.frombuffer(slots, dtype=np.uint8).copy()).to(device)
    z = torch.empty(32 * wc.num_vars, dtype=torch.uint8, device=device)
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t0
    reps = args.winning_reps
    blind = splitmix_frs(6600, 2 * (reps + 3))
    for w in range(2):  # warm-up: program upload, plans, scratch
        wc.witness_dev(ctx, sd.data_ptr(), z.data_ptr())
        fg.prove(ctx, pk, circ, z.data_ptr(), blind[2 * w], blind[2 * w + 1])
    ctx.synchronize()
    ctx.reset_stats()
    lat, proofs = [], []
    for k in range(reps):
        t1 = time.perf_counter()
        wc.witness_dev(ctx, sd.data_ptr(), z.data_ptr())
        proofs.append(fg.prove(ctx, pk, circ, z.data_ptr(), blind[2 * k + 4], blind[2 * k + 5]))
        lat.append(time.perf_counter() - t1)
    st = ctx.stats()
    vk, ic = pk.verifying_key()
    pub = wc.public_inputs(slots)
    verified = bool(fg.verify_batch(vk, ic, [pub] * len(proofs), proofs))
    lat_s = sorted(lat)
    med = lat_s[len(lat_s) // 2]
    n = wc.num_constraints
    out = {"workload": f"Winning PoSt (generate_winning_post) at the reference shape: {wc.sectors} circuit sectors x "
                       f"{wc.challenges} challenge over one replica, 2^{args.winning_log_nodes}-node 8-8-0 tree R-last "
                       f"({n} constraints, {wc.num_inputs} inputs, domain 2^{circ.d.bit_length() - 1}); synthetic "
                       f"consistent replica; timed = GPU witness + proof, one partition per call",
           "constraints": n, "inputs": wc.num_inputs, "domain": circ.d, "reps": reps,
           "latency_ms_median": med * 1e3, "latency_ms_mean": 1e3 * sum(lat) / reps, "latency_ms_min": lat_s[0] * 1e3,
           "constraints_per_s": n / med, "verified": verified, "verified_proofs": len(proofs),
           "device_ms_per_proof": {k: round(st[k]["ms"] / reps, 3) for k in
                                   ("prove", "msm_g1", "msm_g2", "accum_g1", "accum_g2", "sort", "ntt", "wit_a",
                                    "wit_sha", "wit_pos")},
           "setup_s": {"r1cs_build": t_build, "total": t_setup}}
    del pk, circ, z, sd, wc
    gc.collect()
    torch.cuda.synchronize()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--log-rows", type=int, default=26, help="log2 of the evaluation domain (config 3: 26)")
    ap.add_argument("--n-in", type=int, default=4)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--partitions", type=int, default=0,
                    help="config-5 mode: P partitions per step, round-robin over the ranks (0: one per rank)")
    ap.add_argument("--params", default=None,
                    help="load the proving key from a bellman/filecoin params file (mmap) instead of generating it")
    ap.add_argument("--msm-reps", type=int, default=3, help="reps of the standalone 2^log-rows G1 MSM")
    ap.add_argument("--cpu-log-rows", default="21,22,23,24",
                    help="oracle sample sizes (comma-separated log2 rows; >= 3 for the fitted extrapolation)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-device-resident", action="store_true", help="skip the secondary HBM-resident run")
    ap.add_argument("--stats-json", default=None, help="write per-kernel timers here")
    ap.add_argument("--config4-log-rows", type=int, default=27,
                    help="secondary: BASELINE config 4 (2^N domain) after the main run on one GPU (0 skips)")
    ap.add_argument("--config4-steps", type=int, default=2)
    ap.add_argument("--uniform-steps", type=int, default=4,
                    help="one GPU: the headline shape with a uniform witness, timed proofs (0 skips)")
    ap.add_argument("--stacked-log-nodes", type=int, default=30,
                    help="secondary (one GPU): the 32 GiB stacked-PoRep partition witness + prove (0 skips)")
    # default: the 32 GiB PoRep LayerChallenges from select_challenges (11 layers x 18 = ceil(176 / 10) challenges)
    ap.add_argument("--stacked-layers", type=int, default=None)
    ap.add_argument("--stacked-challenges", type=int, default=None)
    ap.add_argument("--stacked-reps", type=int, default=2)
    ap.add_argument("--post-sectors", type=int, default=2349,
                    help="Window-PoSt partition: sectors (0 skips the Window-PoSt / config-5 leg)")
    ap.add_argument("--post-challenges", type=int, default=10)
    ap.add_argument("--post-log-nodes", type=int, default=30)
    ap.add_argument("--post-partitions", type=int, default=10, help="multi-GPU runs: config 5's partition count")
    ap.add_argument("--post-reps", type=int, default=2, help="one GPU: Window-PoSt partitions proven (witness + proof)")
    ap.add_argument("--config5-steps", type=int, default=1)
    ap.add_argument("--post-share-groups", default="4,2",
                    help="one GPU: time the latency-mode shares of one Window-PoSt partition for these group sizes")
    ap.add_argument("--winning-log-nodes", type=int, default=30,
                    help="one GPU: Winning-PoSt latency over a 2^N-node sector (N = 3 (mod 3) for 8-8-0; 0 skips)")
    ap.add_argument("--winning-reps", type=int, default=10)
    ap.add_argument("--tree-log-nodes", type=int, default=21,
                    help="secondary: tree C over 2^N columns x 11 layers (N a multiple of 3; 0 skips)")
    ap.add_argument("--sdr-log-labels", type=int, default=24,
                    help="secondary: SDR labelling-proof labels of 2^N challenges (0 skips)")
    ap.add_argument("--params-roundtrip", type=int, default=1,
                    help="1: write the main key as a params file and time its unchecked / checked load (setup_s)")
    ap.add_argument("--tune", action="append", default=[], metavar="NAME=VALUE",
                    help="library A/B switch for the whole run (mi_tune_set, csrc/tune.h; tools' A/B runs only)")
    args = ap.parse_args()
    if args.stacked_layers is None or args.stacked_challenges is None:
        from fil_groth16.compound import SECTOR_SIZE_32GIB, porep_layer_challenges

        lc = porep_layer_challenges(SECTOR_SIZE_32GIB)
        args.stacked_layers = lc.layers if args.stacked_layers is None else args.stacked_layers
        args.stacked_challenges = lc.max_count if args.stacked_challenges is None else args.stacked_challenges

    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} from the launcher but --gpus "
                             f"{args.gpus}: they must agree")
    elif args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch

    # Multi-rank rehearsal on a one-GPU box (the driver's N > 1 runs use neither): MI_BENCH_BACKEND=gloo
    # keeps the collectives on host tensors and MI_BENCH_SHARED_DEVICE=1 puts every rank on device 0.
    backend = os.environ.get("MI_BENCH_BACKEND", "nccl")
    dev_index = 0 if os.environ.get("MI_BENCH_SHARED_DEVICE") == "1" else local_rank
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(dev_index)
        dist.init_process_group(backend)
    device = torch.device("cuda", dev_index)

    import fil_groth16 as fg

    for kv in args.tune:  # A/B runs of the tools: library switches, never set by the default bench line
        k, _, v = kv.partition("=")
        fg.tune_set(k, int(v))
    from fil_groth16 import synth as synth_mod
    from fil_groth16.compound import shard_partitions
    from fil_groth16.distributed import gather_multiproof, prove_partitions

    t_setup = time.perf_counter()
    ctx = fg.Context(dev_index)
    sc = synth_mod.SynthCircuit(args.log_rows, args.n_in, args.seed)
    t_synth = time.perf_counter() - t_setup
    circ = sc.load(ctx)
    t_load = time.perf_counter() - t_setup - t_synth
    if args.params:
        pk = fg.ProvingKey.load_params(ctx, circ, args.params, checked=False)
    else:
        pk = fg.generate_random_parameters(ctx, circ, splitmix_frs(TOXIC_SEED, 5))
    ctx.synchronize()
    t_srs = time.perf_counter() - t_setup - t_synth - t_load
    free_b, total_b = torch.cuda.mem_get_info(dev_index)
    dev_used_gb = (total_b - free_b) / 1e9  # circuit + proving key (+ split tables unless msm_glv=1)
    # the witness in page-locked host memory, where a synthesiser would write it (mi_host_alloc)
    zhost = fg.HostBuffer(32 * sc.num_vars)
    np.copyto(zhost.array, sc.z_array())
    n = sc.n
    shape = {"d": circ.d, "n_a": circ.n_a, "n_b": circ.n_b, "n_in": sc.n_in, "n_aux": sc.n_aux,
             "num_vars": sc.num_vars}
    vk, ic = pk.verifying_key()
    pub_inputs = zhost.array[32:32 * sc.n_in].tobytes()
    log(rank, f"setup: synth {t_synth:.1f}s circuit load {t_load:.1f}s srs {'load' if args.params else 'gen'} "
              f"{t_srs:.1f}s; n={n} d={circ.d} |a|={circ.n_a} |b|={circ.n_b}")

    # MI_BENCH_PRIORITY=1: the main leg on the context's high-priority stream (lane A/B)
    prio = os.environ.get("MI_BENCH_PRIORITY") == "1"
    P = args.partitions
    mine = shard_partitions(P, rank, world) if P else [rank]
    per_step = len(mine)
    blind = splitmix_frs(1000, 2 * (args.warmup + args.steps) * max(P, world))

    def blinding(step, part):
        i = step * max(P, world) + part
        return blind[2 * i], blind[2 * i + 1]

    if args.warmup:
        fg.prove_batch(ctx, pk, circ, [zhost] * (args.warmup * per_step),
                       [blinding(w, p) for w in range(args.warmup) for p in mine], priority=prio)
    ctx.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.reset_stats()

    gdev = device if dist and backend == "nccl" else "cpu"
    t0 = time.perf_counter()
    if P:
        multiproofs = []
        for k in range(args.steps):
            step = args.warmup + k
            multiproofs.append(prove_partitions(
                lambda ids: fg.prove_batch(ctx, pk, circ, [zhost] * len(ids), [blinding(step, p) for p in ids],
                                           priority=prio),
                P, rank, world, gdev))
        proofs = [mp_[192 * i:192 * (i + 1)] for mp_ in multiproofs for i in range(P)]
    else:
        # K partitions of this rank in one batch: partition k + 1's upload overlaps proof k
        local = fg.prove_batch(ctx, pk, circ, [zhost] * args.steps,
                               [blinding(args.warmup + k, rank) for k in range(args.steps)], priority=prio)
        # MultiProof assembly: every rank's proofs gathered in (step, rank) order over RCCL
        proofs = gather_multiproof(local, args.steps * world, rank, world, gdev) if dist else b"".join(local)
        proofs = [proofs[192 * i:192 * (i + 1)] for i in range(len(proofs) // 192)]
    ctx.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([dt], dtype=torch.float64, device=gdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    stats = ctx.stats()
    proofs_total = args.steps * (P if P else world)

    # the C2 self-check policy (api/seal.hpp:310-313), outside the timer: every gathered proof is
    # pairing-verified (one batch multi-pairing with OS-random weights) and the last one singly
    log(rank, f"main leg: {1e3 * dt / args.steps:.1f} ms per step, {proofs_total} proofs")
    t_ver = time.perf_counter()
    verified = bool(fg.verify_batch(vk, ic, [pub_inputs] * len(proofs), proofs)) and \
        bool(fg.verify(vk, ic, pub_inputs, proofs[-1]))
    t_ver = time.perf_counter() - t_ver

    # secondary: the same proof with the witness already resident in HBM (no upload)
    resident = None
    if not args.no_device_resident:
        zdev = torch.from_numpy(sc.z_array().copy()).to(device)
        k2 = max(2, args.steps // 4)
        fg.prove(ctx, pk, circ, zdev.data_ptr(), *blinding(0, 0))
        ctx.synchronize()
        tr = time.perf_counter()
        for k in range(k2):
            fg.prove(ctx, pk, circ, zdev.data_ptr(), *blinding(k, 0))
        ctx.synchronize()
        tr = (time.perf_counter() - tr) / k2
        resident = {"value": n / tr, "unit": "constraints/s", "ms_per_proof": tr * 1e3, "proofs": k2,
                    "note": "witness resident in HBM before the timer (no H2D): the round-1 definition"}
        del zdev

    # the dominant kernel measured alone: one proof with prove_lanes=1 (the auxiliary lane's MSMs run after the
    # main lane's, on the same stream), so k_accum_level0's launch times are the kernel's own and not stretched by
    # the other lane's sorts and NTTs (the timed proofs' two-lane figure is reported beside it)
    one_lane = None
    a_plan = None  # how this key's proofs plan A's MSM: "own", "shared" (one plan with L) or "derived" (from L's)
    if rank == 0:
        try:
            with fg.tuned(prove_lanes=1):
                ctx.reset_stats()
                fg.prove_batch(ctx, pk, circ, [zhost], [blinding(0, 0)], priority=prio)
                ctx.synchronize()
            one_lane = ctx.stats()
            a_plan = "derived" if ctx.derived_plans() else "shared" if ctx.shared_plans() else "own"
        except Exception as e:  # reported, never fatal
            one_lane = {"error": str(e)}

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
        # the same 2^20 fixed bases with a window table (mi_points_precompute: T[w n + i] = 2^(c w) P_i, built once
        # outside the timer, as a key's small queries carry theirs): one bucket set for every window
        tb = time.perf_counter()
        pts.precompute(0, m20)
        ctx.synchronize()
        tb = time.perf_counter() - tb
        tinfo = pts.table_info()
        pts.msm_dev(sc_dev.data_ptr(), m20)
        ctx.synchronize()
        tm = time.perf_counter()
        for _ in range(10):
            pts.msm_dev(sc_dev.data_ptr(), m20)
        ctx.synchronize()
        t20w = (time.perf_counter() - tm) / 10
        micro = {"workload": "BASELINE configs[1]: 2^20-point G1 MSM + 2^20-element Fr NTT, device-resident",
                 "msm_g1_2e20_ms": t20 * 1e3, "msm_g1_2e20_mpoints_per_s": m20 / t20 / 1e6,
                 "msm_g1_2e20_table_ms": t20w * 1e3, "msm_g1_2e20_table_mpoints_per_s": m20 / t20w / 1e6,
                 "table": dict(tinfo, build_ms=tb * 1e3, gbytes=tinfo["points"] * tinfo["windows"] * 128 / 1e9,
                               note="fixed-base window table of the 2^20 bases (built once, outside the timer); "
                                    "msm_g1_2e20_* is the same MSM without it"),
                 "ntt_fr_2e20_ms": n20 * 1e3, "ntt_fr_2e20_melems_per_s": m20 / n20 / 1e6}
        del x
    del sc_dev, pts

    # the key load every prover process does once per shape (get_groth_params -> read_cached_params ->
    # build_mapped_parameters, core/parameter_cache.hpp:124-128,185-200; mmap at mapped_scheme_params.hpp:50-60): the
    # main key written as a v28 params file, loaded back unchecked and subgroup-checked (mi_params_load), and the
    # loaded key's proof compared with the resident key's, outside every timer
    params_load = None
    if rank == 0 and world == 1 and args.params_roundtrip and not args.params:
        try:
            params_load = params_roundtrip(fg, ctx, circ, pk, zhost, blinding(0, 0))
        except Exception as e:  # reported, never fatal
            params_load = {"error": str(e)}
        log(rank, f"params round trip: {params_load}")

    # tree C over one 2^tree_log_nodes-node sub-tree (device-resident labels), and the
    # oracle's CPU Poseidon on a sample of the same columns
    log(rank, "secondary: MSM / configs[1] micro done")
    tree = None
    if args.tree_log_nodes and rank == 0:
        tree = tree_c_leg(args, fg, ctx, device, world)
        log(rank, "tree C leg done")

    # SDR labelling-witness labels (SHA-256 over gathered parents)
    sdr = None
    if args.sdr_log_labels and rank == 0:
        try:
            sdr = sdr_leg(args, fg, ctx, device, world)
        except Exception as e:  # reported, never fatal to the main measurement
            sdr = {"error": str(e)}
        log(rank, "SDR label leg done")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args, fg, synth_mod, ctx)
        except Exception as e:  # reported, never fatal to the GPU measurement
            cpu = {"value": None, "unit": "constraints/s", "cores": None, "kind": "port", "sample": f"failed: {e}"}

    config5 = None
    if world > 1 and not P and args.post_sectors:
        import gc

        del pk, circ, zhost, sc
        gc.collect()
        ctx.synchronize()
        try:
            log(rank, "config 5 leg (Window-PoSt partitions) ...")
            config5 = window_post_leg(args, fg, ctx, device, rank, world, gdev, dist)
        except Exception as e:  # reported, never fatal to the main measurement
            config5 = {"error": str(e)}

    if rank == 0 and world == 1 and (args.config4_log_rows or args.stacked_log_nodes or args.post_sectors or
                                     args.winning_log_nodes or args.uniform_steps):
        import gc

        del pk, circ, zhost, sc  # the secondary legs need the HBM
        gc.collect()
        ctx.synchronize()
    uniform = None
    if rank == 0 and world == 1 and args.uniform_steps:
        try:
            log(rank, "uniform-witness leg ...")
            uniform = uniform_leg(args, fg, synth_mod, ctx)
        except Exception as e:  # reported, never fatal to the config-3 measurement
            uniform = {"value": None, "error": str(e)}

    config4 = None
    if rank == 0 and world == 1 and args.config4_log_rows:
        try:
            log(rank, "config 4 leg ...")
            config4 = config4_leg(args, fg, synth_mod, ctx)
        except Exception as e:  # reported, never fatal to the config-3 measurement
            config4 = {"value": None, "error": str(e)}

    stacked_res = None
    if rank == 0 and world == 1 and args.stacked_log_nodes:
        try:
            log(rank, "stacked PoRep leg ...")
            stacked_res = stacked_leg(args, fg, ctx, device, world)
        except Exception as e:  # reported, never fatal to the config-3 measurement
            stacked_res = {"error": str(e)}

    winning = None
    if rank == 0 and world == 1 and args.winning_log_nodes:
        try:
            log(rank, "Winning-PoSt leg ...")
            winning = winning_post_leg(args, fg, ctx, device)
        except Exception as e:  # reported, never fatal to the config-3 measurement
            winning = {"error": str(e)}

    post_res = None
    if rank == 0 and world == 1 and args.post_sectors and args.post_reps:
        try:
            log(rank, "Window-PoSt leg ...")
            post_res = window_post_leg(args, fg, ctx, device, rank, world, None, None)
        except Exception as e:  # reported, never fatal to the config-3 measurement
            post_res = {"error": str(e)}

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
    # HBM traffic of the dominant kernel from the committed rocprofv3 PMC summary of the same workload (FETCH_SIZE
    # and WRITE_SIZE passes, per point): bytes per launch = per-point bytes x points per launch, and as a rate
    # over this run's average launch time (GB/s, the unit of `achieved`).  Raw FETCH_SIZE and the gfx950 x2
    # correction (MI355X_MICROARCH.md) are reported separately; `traffic` is the corrected rate, an upper bound
    # for this gather-bound kernel.
    traffic, traffic_detail = None, None
    prof_dir = os.path.join(ROOT, "profiles")
    if os.path.isdir(prof_dir):
        for fn in sorted(os.listdir(prof_dir), reverse=True):
            if fn.endswith("_summary.json"):
                try:
                    ps = json.load(open(os.path.join(prof_dir, fn)))
                    dk = ps.get("dominant_kernel", {})
                    if grp == "G1" and "hbm_bytes_per_point" in dk and ps.get("workload") == \
                            workload_name(args.log_rows):
                        wr = dk.get("write_bytes_per_point", 0.0)
                        raw_b = (dk.get("fetch_bytes_raw_per_point", 0.0) + wr) * units_per_launch
                        cor_b = dk["hbm_bytes_per_point"] * units_per_launch
                        sec = avg_ms * 1e-3
                        traffic = cor_b / sec / 1e9 if sec > 0 else None
                        traffic_detail = {
                            "unit": "GB/s", "bytes_per_launch_raw": raw_b, "bytes_per_launch_corrected": cor_b,
                            "gbps_raw": raw_b / sec / 1e9 if sec > 0 else None, "gbps_corrected": traffic,
                            "bytes_per_point_raw": raw_b / units_per_launch if units_per_launch else None,
                            "bytes_per_point_corrected": dk["hbm_bytes_per_point"],
                            "source": f"profiles/{fn}", "profiled_at_commit": ps.get("commit"),
                            "profiled_launch_avg_ms": dk.get("timed_step_launch_avg_ms"),
                            "note": "FETCH_SIZE (+ WRITE_SIZE) per point from separate --pmc passes x points per "
                                    "launch of this run; corrected = FETCH x 2 (gfx950, stated for streaming "
                                    "reads; an upper bound for these 128-B record gathers), rate over this run's "
                                    "average launch time"}
                        break
                except Exception:
                    pass
    # secondary (binding) roofline: Fq multiplications per second vs the MAD-issue bound, over the mixed
    # additions the accumulation actually issued (non-zero signed digits, counted by the library)
    madds_per_launch = dom.get("madds", 0) / max(dom["launches"], 1)
    # the ceiling of the kernel's own group law on this chip: the maddloop microbenchmark's gathered-record
    # rate for the library's record layout (microbench/maddloop.hip; in-kernel clock, two waves per SIMD)
    ceiling = None
    if os.path.isdir(prof_dir) and grp == "G1":
        for fn in sorted(os.listdir(prof_dir), reverse=True):
            if "_maddloop" in fn and fn.endswith(".jsonl"):  # the newest round's microbenchmark with the gather128 form
                rows = [json.loads(l) for l in open(os.path.join(prof_dir, fn)) if l.strip().startswith("{")]
                g = [r for r in rows if r.get("form") == "gather128"]
                if g:
                    ceiling = {"source": f"profiles/{fn}", "form": "gather128 (the library's padded 128-byte records)",
                               "gmadd_per_s": max(r["gmadd_per_s"] for r in g),
                               "clock_ghz": max(r["clock_ghz_median"] for r in g)}
                    break
    one_lane_res = None
    if one_lane and "accum_g1" in one_lane and grp == "G1" and one_lane["accum_g1"]["launches"]:
        o = one_lane["accum_g1"]
        o_ms = o["ms"] / o["launches"]
        o_madds = o.get("madds", 0) / o["launches"]
        o_rate = o_madds / (o_ms * 1e-3) / 1e9 if o_ms > 0 else None
        one_lane_res = {
            "mode": "one lane (prove_lanes=1, one proof): the kernel alone on the chip",
            "avg_launch_ms": o_ms, "launches": o["launches"], "madds_per_launch": o_madds, "gmadd_per_s": o_rate,
            "hbm_frac": (bytes_per_unit * o["units"] / o["launches"] / (o_ms * 1e-3) / 1e9) / HBM_PEAK_GBS
            if o_ms > 0 else None,
            "group_law_ceiling_frac": o_rate / ceiling["gmadd_per_s"] if ceiling and o_rate else None,
            "proof_ms": one_lane["prove"]["ms"] / max(one_lane["prove"]["launches"], 1)}
    fq_muls = madds_per_launch * FQ_MUL_PER_MIXED_ADD[grp]
    valu_ach = fq_muls / (avg_ms * 1e-3) if avg_ms > 0 and fq_muls else None
    valu_peak = MAD_RATE / FQ_MUL_MADS
    value = n * proofs_total / dt
    h2d = stats["h2d"]
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
        "data": "synthetic R1CS + satisfying witness (csrc/synth.hip) in page-locked host memory, proving key "
                + ("loaded from " + args.params if args.params else "generated on device from fixed toxic waste"),
        "config": {"workload": workload_name(args.log_rows, P, world),
                   "constraints": n, "domain": shape["d"], "num_inputs": shape["n_in"], "num_aux": shape["n_aux"],
                   "a_query": shape["n_a"], "b_query": shape["n_b"], "proofs_per_step": P if P else world,
                   "partitions_per_rank": per_step, "a_plan": a_plan,
                   "parallelism": f"partition-sharded x{world}"},
        "verified": verified,
        "verified_proofs": len(proofs),
        "verify_s": t_ver,
        "witness": "host (pinned), H2D of partition k + 1 overlapped with proof k",
        "h2d": {"ms_per_proof": h2d["ms"] / max(h2d["launches"], 1),
                "gb_per_s": h2d["units"] / max(h2d["ms"], 1e-9) / 1e6, "bytes_per_proof": 32 * shape["num_vars"]},
        "device_resident": resident,
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
            "traffic_unit": "GB/s",
            "traffic_detail": traffic_detail,
            "avg_launch_ms": avg_ms,
            "units_per_launch": units_per_launch,
            "algorithmic_bytes_per_unit": bytes_per_unit,
            "note": "VALU-integer-bound kernel (BLS12-381 Montgomery multiplications); HBM fraction is reported "
                    "per BASELINE.json north_star; the binding roofline is 'valu_roofline'",
        },
        "valu_roofline": {
            "bound": "valu (v_mad_i64_i32 issue)",
            "kernel": dom_name,
            "achieved": valu_ach,
            "peak": valu_peak,
            "unit": "Fq-mul/s",
            "frac": valu_ach / valu_peak if valu_ach else None,
            "madds_per_launch": madds_per_launch,
            "group_law_ceiling": dict(ceiling, frac=(madds_per_launch / (avg_ms * 1e-3) / 1e9) / ceiling["gmadd_per_s"],
                                      frac_is="two lanes: the timed proofs' launches, stretched by the other lane's "
                                              "sorts and NTTs sharing the CUs")
            if ceiling and avg_ms > 0 and madds_per_launch else None,
            "one_lane": one_lane_res,
            "spec_issue": {"peak_lane_instr_per_s": SPEC_VALU_LANE_INSTR,
                           "instr_per_mixed_add": G1_MADD_VALU_INSTR if grp == "G1" else None,
                           "frac": (madds_per_launch * G1_MADD_VALU_INSTR / (avg_ms * 1e-3) / SPEC_VALU_LANE_INSTR)
                           if grp == "G1" and avg_ms > 0 and madds_per_launch else None,
                           "note": "ISA VALU instructions per mixed add x mixed adds issued / launch time, against "
                                   "the spec issue rate (MI355X_MICROARCH.md: 32 lanes/cycle/SIMD); the gap to "
                                   "1 is the MAD's 4-cycle issue (measured, DESIGN.md §5) and DVFS"},
            "model": f"{FQ_MUL_PER_MIXED_ADD[grp]} Fq-mul per mixed add x mixed adds issued (non-zero signed digits "
                     f"counted by the library; split-mode MSMs: 2n half-scalar points over 6 windows); "
                     f"peak = v_mad_i64_i32 issue rate / {FQ_MUL_MADS} MADs",
        },
        "cpu_baseline": cpu,
        "tree_c": tree,
        "sdr_labels": sdr,
        "uniform_witness": uniform,
        "config4": config4,
        "config5": config5,
        "stacked_porep_32gib": stacked_res,
        "window_post_32gib": post_res,
        "winning_post_32gib": winning,
        "timers_ms": {k: round(v["ms"], 3) for k, v in stats.items()},
        "setup_s": {"synth": t_synth, "circuit_load": t_load, "srs": t_srs, "params_load": params_load},
        "device_gb_after_setup": round(dev_used_gb, 2),
        "msm_split": {1: "glv", 0: "2^128 tables"}.get(fg.tune_get("msm_glv"),
                                                      "auto: 2^128 tables when they fit in HBM, else glv"),
        "tune": args.tune,
        "multiproof_bytes": 192 * len(proofs),
        "msm_reps": args.msm_reps,
    }
    if cpu and cpu.get("value"):
        out["gpu_over_cpu"] = value / cpu["value"]
        if cpu.get("extrapolated"):
            out["gpu_over_cpu_extrapolated_same_size"] = value / cpu["extrapolated"]["constraints_per_s"]
    if args.stats_json:
        with open(args.stats_json, "w") as f:
            json.dump(stats, f, indent=1)
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
