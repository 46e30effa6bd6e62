"""GPU parity for the full Groth16 prover (crypto3 r1cs_gg_ppzksnark / bellman semantics).

* golden fixtures: the SRS from the oracle's keygen is loaded through mi_srs_load and the proof
  must equal the fixture bytes (which the independent Python restatement produced and a pairing
  check accepted);
* GPU parameter generation (mi_srs_generate) must reproduce the oracle keygen query-for-query;
* larger circuits: GPU proof == oracle proof, oracle pairing verifier accepts it;
* BASELINE-size property: trapdoor discrete logs of (A, B, C) at 2^20 constraints.
"""
import numpy as np
import pytest

import circuits
import fil_groth16 as fg

pytestmark = pytest.mark.gpu


def _circuit_from_name(name):
    if name.startswith("random"):
        _, seed, rows = name.split("_")
        return circuits.random_circuit(int(seed), int(rows))
    return circuits.toy_chain(1022)


def _load(ctx, oracle, n_in, n_aux, rows, z):
    mats = circuits.to_csr(rows)
    oc = oracle.OracleCircuit(len(rows), n_in, n_aux, mats)
    gc = fg.Circuit(ctx, len(rows), n_in, n_aux, mats)
    return oc, gc


@pytest.mark.parametrize("name", ["random_11_24", "random_12_60", "toy_chain_1022"])
def test_groth16_golden_loaded_srs(ctx, oracle, golden, name):
    g = golden["groth16"][name]
    n_in, n_aux, rows, z = _circuit_from_name(name)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rows, z)
    op = oracle.OracleParams(oc, circuits.toxic())
    ex = op.export()
    pk = fg.ProvingKey.load(ctx, gc, ex["vk"], ex["ic"], ex["h"], ex["l"], ex["a"], ex["b_g1"], ex["b_g2"],
                            checked=True)
    r, s = circuits.blinding()
    proof, raw = fg.prove(ctx, pk, gc, circuits.z_bytes(z), r, s, want_raw=True)
    assert proof.hex() == g["proof"]
    assert raw.hex() == g["raw"]


@pytest.mark.parametrize("name", ["random_11_24", "random_12_60", "toy_chain_1022"])
def test_groth16_golden_generated_srs(ctx, oracle, golden, name):
    g = golden["groth16"][name]
    n_in, n_aux, rows, z = _circuit_from_name(name)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rows, z)
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    op = oracle.OracleParams(oc, circuits.toxic())
    ex = op.export()
    assert [pk.n_h, pk.n_l, pk.n_a, pk.n_b, pk.n_b] == g["query_sizes"]
    vk, ic = pk.verifying_key()
    assert vk == ex["vk"] and ic == ex["ic"]
    for which, key in enumerate(("h", "l", "a", "b_g1", "b_g2")):
        assert pk.query(which) == ex[key], key
    r, s = circuits.blinding()
    assert fg.prove(ctx, pk, gc, circuits.z_bytes(z), r, s).hex() == g["proof"]


def test_groth16_unsatisfied_witness_matches_oracle(ctx, oracle):
    """Bit-exactness does not depend on satisfiability (the prover is a deterministic map)."""
    n_in, n_aux, rows, z = circuits.random_circuit(21, 40)
    z = list(z)
    z[-1] = (z[-1] + 1) % fg.FR_MODULUS
    oc, gc = _load(ctx, oracle, n_in, n_aux, rows, z)
    op = oracle.OracleParams(oc, circuits.toxic())
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    zb = circuits.z_bytes(z)
    r, s = 5, 7
    assert fg.prove(ctx, pk, gc, zb, r, s) == op.prove(zb, r, s)[0]


@pytest.mark.parametrize("rows,seed", [(700, 31), (5000, 32), (16000, 33)])
def test_groth16_random_vs_oracle_and_pairing(ctx, oracle, rows, seed):
    n_in, n_aux, rws, z = circuits.random_circuit(seed, rows, n_in=6, n_free=32)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rws, z)
    tox = circuits.toxic(seed)
    pk = fg.generate_random_parameters(ctx, gc, tox)
    op = oracle.OracleParams(oc, tox)
    zb = circuits.z_bytes(z)
    r, s = circuits.blinding(seed)
    proof, raw = fg.prove(ctx, pk, gc, zb, r, s, want_raw=True)
    oproof, oraw, _ = op.prove(zb, r, s)
    assert proof == oproof and raw == oraw
    vk, ic = pk.verifying_key()
    assert oracle.groth16_verify(vk, ic, zb[:32 * n_in], raw)
    assert op.trapdoor_check(zb, r, s, raw)
    # zero blinding edge case (r = s = 0) still matches
    assert fg.prove(ctx, pk, gc, zb, 0, 0) == op.prove(zb, 0, 0)[0]


def test_groth16_windowed_sort_vs_oracle(ctx, oracle, tune):
    """The large-MSM paths of a prove (per-window sort of the compacted non-zero digits, the B_G1 / B_G2
    plan shared in that mode, G2 second-level bucket reduction), forced at a size the oracle proves in
    seconds."""
    tune.set("msm_sort", 1 if "windowed" == "windowed" else 0)
    tune.set("g2_l2", 2)  # and B_G2's bucket reduction as the second-level MSM
    n_in, n_aux, rws, z = circuits.random_circuit(34, 5000, n_in=6, n_free=32)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rws, z)
    tox = circuits.toxic(34)
    pk = fg.generate_random_parameters(ctx, gc, tox)
    op = oracle.OracleParams(oc, tox)
    zb = circuits.z_bytes(z)
    r, s = circuits.blinding(34)
    proof, raw = fg.prove(ctx, pk, gc, zb, r, s, want_raw=True)
    oproof, oraw, _ = op.prove(zb, r, s)
    assert proof == oproof and raw == oraw


@pytest.mark.parametrize("split", ["0", "2", "glv"])
def test_groth16_split_msm_vs_oracle(ctx, oracle, tune, split):
    """H, L and A through the split-mode MSM (2^128 base tables, two 128-bit half scalars per point)
    forced at a size the oracle proves in seconds; "0" is the plain path at the same size, "glv" the
    split through the GLV endomorphism (no tables built at key generation)."""
    tune.set("msm_split", int("2" if split == "glv" else split))
    tune.set("msm_glv", int("1" if split == "glv" else "0"))
    tune.set("msm_wt_max_log", 0)  # this key's MSMs on the split / plain paths, not window tables
    n_in, n_aux, rws, z = circuits.random_circuit(35, 5000, n_in=6, n_free=32)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rws, z)
    tox = circuits.toxic(35)
    pk = fg.generate_random_parameters(ctx, gc, tox)
    op = oracle.OracleParams(oc, tox)
    zb = circuits.z_bytes(z)
    r, s = circuits.blinding(35)
    assert fg.prove(ctx, pk, gc, zb, r, s) == op.prove(zb, r, s)[0]
    vk, _ = pk.verifying_key()
    shares = [fg.prove_share(ctx, pk, gc, zb, k, 3) for k in range(3)]  # latency-mode slices, same path
    assert fg.assemble(vk, shares, r, s) == op.prove(zb, r, s)[0]


@pytest.mark.parametrize("n_in,cover", [(2, 1.0), (6, 0.96), (300, 1.0), (6, 0.5)])
def test_groth16_shared_la_plan_vs_oracle(ctx, oracle, tune, n_in, cover):
    """VERDICT r5 #1b: a large subgroup key whose A density covers >= 90 % of the aux variables holds its A query in the
    aux index space (mi_srs_shared_la), so a whole proof's L and A MSMs run over ONE GLV plan -- built on the
    auxiliary lane, L accumulated there, A's aux part on the main lane after H, the inputs' part of A as a small MSM
    -- and the proof equals the oracle's byte for byte.  Forced at a size the oracle proves in seconds (split at any
    size, no window tables, the two-lane layout of large proofs).  random_circuit's later outputs rarely appear in an
    A term, so rows "v * 0 = 0" give a fraction `cover` of those variables A density; the rest sit at infinity in
    the gathered query.  One lane, latency-mode shares (separate plans over ranges), an all-zero aux witness and an
    out-of-memory retry (which drops the gathered query: separate plans again) give the same bytes.  cover = 0.5
    stays below the admission rule: separate plans, as before."""
    tune.set("msm_split", 2)
    tune.set("msm_wt_max_log", 0)
    tune.set("prove_wide_log", 0)
    n_in_, n_aux, rws, z = circuits.random_circuit(37 + n_in, 3000, n_in=n_in, n_free=32)
    in_a = {c for row in rws for c, _ in row[0]}
    missing = [v for v in range(n_in_, n_in_ + n_aux) if v not in in_a]
    rws = rws + [([(v, 1)], [], []) for v in missing[:int(cover * len(missing))]]
    dense = sum(1 for v in range(n_in_, n_in_ + n_aux) if v in in_a) + int(cover * len(missing))
    oc, gc = _load(ctx, oracle, n_in_, n_aux, rws, z)
    tox = circuits.toxic(37)
    pk = fg.generate_random_parameters(ctx, gc, tox)
    assert pk.shared_la() == (dense * 10 >= n_aux * 9)
    op = oracle.OracleParams(oc, tox)
    zb = circuits.z_bytes(z)
    want = op.prove(zb, 5, 6)[0]
    ctx.reset_stats()
    assert fg.prove(ctx, pk, gc, zb, 5, 6) == want
    shared = 1 if pk.shared_la() else 0
    assert ctx.shared_plans() == shared
    tune.set("prove_lanes", 1)
    assert fg.prove(ctx, pk, gc, zb, 5, 6) == want
    tune.clear("prove_lanes")
    assert ctx.shared_plans() == 2 * shared
    vk, _ = pk.verifying_key()
    assert fg.assemble(vk, [fg.prove_share(ctx, pk, gc, zb, k, 2) for k in range(2)], 5, 6) == want
    assert ctx.shared_plans() == 2 * shared  # shares run over ranges: plans of their own
    zeros = zb[:32 * n_in_] + bytes(32 * n_aux)  # every aux scalar zero: an empty shared plan
    assert fg.prove(ctx, pk, gc, zeros, 5, 6) == op.prove(zeros, 5, 6)[0]
    ctx.inject_oom(1)
    assert fg.prove(ctx, pk, gc, zb, 7, 8) == op.prove(zb, 7, 8)[0]
    assert not pk.shared_la() and ctx.fallbacks()["oom_retries"] == 1


@pytest.mark.parametrize("mode", ["tables", "glv", "short_chunks"])
def test_groth16_derived_a_plan_vs_oracle(ctx, oracle, tune, mode):
    """Keys below the shared plan's density rule: L's plan carries A's density in its entries and A's plan is filtered
    out of it (msm_derive_plan: no digit pass, no sort of its own), on the lane that runs L, then accumulated over A's
    own points on the main lane.  Over the 2^128 split tables and over GLV; both auxiliary-lane orders, one lane, an
    all-zero aux witness (empty plans), A's own plan (a_from_l = 0), and latency-mode shares (ranges: plans of their
    own) give the oracle's bytes."""
    tune.set("msm_split", 2)
    tune.set("msm_wt_max_log", 0)
    tune.set("prove_wide_log", 0)
    if mode == "glv":
        tune.set("msm_glv", 1)
    if mode == "short_chunks":  # level-0 chunks of 2 entries, 4 partials per tree thread: every derived bucket of
        tune.set("msm_l0", 2)   # 3+ entries goes through the multi-chunk list and chunk-tree levels of its own slots
        tune.set("msm_l1", 4)
    n_in, n_aux, rws, z = circuits.random_circuit(41, 3000, n_in=3, n_free=32)
    in_a = {c for row in rws for c, _ in row[0]}
    assert sum(1 for v in range(n_in, n_in + n_aux) if v in in_a) * 10 < n_aux * 9  # below the shared-plan rule
    oc, gc = _load(ctx, oracle, n_in, n_aux, rws, z)
    tox = circuits.toxic(41)
    pk = fg.generate_random_parameters(ctx, gc, tox)
    assert not pk.shared_la()
    op = oracle.OracleParams(oc, tox)
    zb = circuits.z_bytes(z)
    want = op.prove(zb, 5, 6)[0]
    ctx.reset_stats()
    assert fg.prove(ctx, pk, gc, zb, 5, 6) == want
    assert ctx.derived_plans() == 1 and ctx.shared_plans() == 0
    tune.set("aux_order", 1)  # L (and the derived plan) before B on the auxiliary lane
    assert fg.prove(ctx, pk, gc, zb, 5, 6) == want
    tune.clear("aux_order")
    tune.set("prove_lanes", 1)
    assert fg.prove(ctx, pk, gc, zb, 5, 6) == want
    tune.clear("prove_lanes")
    assert ctx.derived_plans() == 3
    tune.set("a_from_l", 0)
    assert fg.prove(ctx, pk, gc, zb, 5, 6) == want
    tune.clear("a_from_l")
    assert ctx.derived_plans() == 3
    vk, _ = pk.verifying_key()
    assert fg.assemble(vk, [fg.prove_share(ctx, pk, gc, zb, k, 2) for k in range(2)], 5, 6) == want
    assert ctx.derived_plans() == 3
    zeros = zb[:32 * n_in] + bytes(32 * n_aux)
    assert fg.prove(ctx, pk, gc, zeros, 5, 6) == op.prove(zeros, 5, 6)[0]
    # only the inputs and the variables without A density non-zero: A's derived plan is empty, L's is not
    zl = bytearray(zb)
    for v in range(n_in, n_in + n_aux):
        if v in in_a:
            zl[32 * v:32 * v + 32] = bytes(32)
    assert fg.prove(ctx, pk, gc, bytes(zl), 5, 6) == op.prove(bytes(zl), 5, 6)[0]
    assert ctx.derived_plans() == 5


def test_prove_out_of_memory_degrades_to_glv(ctx, oracle, tune):
    """A proof whose scratch allocation fails (mi_ctx_inject_oom, a test-only entry: the main lane raises
    hipMalloc's out-of-memory error after the NTT chain while the auxiliary lane runs) is re-run in-process after
    the key's 2^128 split tables are released: the bytes equal the oracle's, the key reports no tables afterwards,
    and the context counts the retry.  Every prove entry (host / device witness, batch, share) recovers alike.
    mi_srs_readmit then rebuilds the tables (the release is not one-way) and the proof is unchanged."""
    tune.set("msm_split", 2)  # split mode at this size, so the tables are in use
    tune.set("msm_wt_max_log", 0)  # split tables, not window tables
    n_in, n_aux, rws, z = circuits.random_circuit(36, 5000, n_in=6, n_free=32)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rws, z)
    tox = circuits.toxic(36)
    pk = fg.generate_random_parameters(ctx, gc, tox)
    assert pk.msm_info() == {"split_tables": True, "subgroup": True}
    op = oracle.OracleParams(oc, tox)
    zb = circuits.z_bytes(z)
    want = [op.prove(zb, 10 + k, 20 + k)[0] for k in range(3)]
    assert fg.prove(ctx, pk, gc, zb, 10, 20) == want[0]
    ctx.reset_stats()
    ctx.inject_oom(1)
    assert fg.prove(ctx, pk, gc, zb, 10, 20) == want[0]
    fb = ctx.fallbacks()
    assert fb["oom_retries"] == 1 and fb["freed_bytes"] > 0
    assert pk.msm_info() == {"split_tables": False, "subgroup": True}
    assert pk.table_state() == {"split_tables": False, "dropped": 1, "subgroup": True}
    ctx.inject_oom(-1)
    import torch

    zd = torch.from_numpy(np.frombuffer(zb, dtype=np.uint8).copy()).cuda()
    assert fg.prove(ctx, pk, gc, zd.data_ptr(), 11, 21) == want[1]
    assert fg.prove_batch(ctx, pk, gc, [zb, zb], [(10, 20), (12, 22)]) == [want[0], want[2]]
    vk, _ = pk.verifying_key()
    assert fg.assemble(vk, [fg.prove_share(ctx, pk, gc, zb, k, 2) for k in range(2)], 10, 20) == want[0]
    assert ctx.fallbacks()["oom_retries"] == 6
    ctx.inject_oom(0)
    ctx.reset_stats()
    assert fg.prove(ctx, pk, gc, zb, 12, 22) == want[2] and ctx.fallbacks()["oom_retries"] == 0
    # re-admission: the tables come back once they fit, and the proofs keep their bytes
    assert pk.readmit() > 0
    assert pk.table_state() == {"split_tables": True, "dropped": 0, "subgroup": True}
    assert pk.readmit() == 0  # nothing to rebuild
    assert fg.prove(ctx, pk, gc, zb, 11, 21) == want[1] and ctx.fallbacks()["oom_retries"] == 0


def test_prove_window_tables(ctx, oracle, tune):
    """A small key builds fixed-base window tables for h, l, a, b_g1 and b_g2 at generation (domain <= 2^21): its
    proofs run those five MSMs over one bucket set each and equal the oracle's, as do latency-mode shares (table slices at
    an offset); msm_wt=0 (the plain path) gives the same bytes.  An out-of-memory retry releases the tables like
    the split tables, and mi_srs_readmit rebuilds them."""
    tune.clear("msm_wt_max_log")
    tune.clear("msm_wt")
    n_in, n_aux, rws, z = circuits.random_circuit(37, 6000, n_in=5, n_free=40)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rws, z)
    tox = circuits.toxic(37)
    pk = fg.generate_random_parameters(ctx, gc, tox)
    wt = pk.window_tables()
    assert wt["queries"] == 5 and wt["windows"] == -(-256 // wt["window_bits"]), wt
    op = oracle.OracleParams(oc, tox)
    zb = circuits.z_bytes(z)
    want = [op.prove(zb, 30 + k, 40 + k)[0] for k in range(2)]
    ctx.reset_stats()
    assert fg.prove(ctx, pk, gc, zb, 30, 40) == want[0]
    assert ctx.table_msms() == 4 and ctx.table_msms(g2=True) == 1
    vk, _ = pk.verifying_key()
    assert fg.assemble(vk, [fg.prove_share(ctx, pk, gc, zb, k, 3) for k in range(3)], 31, 41) == want[1]
    tune.set("msm_wt", 0)
    ctx.reset_stats()
    assert fg.prove(ctx, pk, gc, zb, 31, 41) == want[1] and ctx.table_msms() == 0 and ctx.table_msms(g2=True) == 0
    tune.clear("msm_wt")
    ctx.inject_oom(1)
    assert fg.prove(ctx, pk, gc, zb, 30, 40) == want[0]
    assert ctx.fallbacks()["oom_retries"] == 1
    assert pk.window_tables()["queries"] == 0 and pk.table_state()["dropped"] == 1
    assert pk.readmit() > 0
    assert pk.window_tables() == wt
    ctx.reset_stats()
    assert fg.prove(ctx, pk, gc, zb, 31, 41) == want[1] and ctx.table_msms() == 4


def test_prove_batch_and_priority(ctx, oracle):
    n_in, n_aux, rws, z = circuits.random_circuit(41, 300)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rws, z)
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    op = oracle.OracleParams(oc, circuits.toxic())
    zb = circuits.z_bytes(z)
    rs = [(1, 2), (3, 4), (5, 6)]
    proofs = fg.prove_batch(ctx, pk, gc, [zb] * 3, rs, priority=True)
    for p, (r, s) in zip(proofs, rs):
        assert p == op.prove(zb, r, s)[0]
    mp = fg.MultiProof(proofs)
    assert fg.MultiProof.from_bytes(mp.to_bytes()).circuit_proofs == proofs


def test_prove_lane_layouts_identical(ctx, oracle, tune):
    """Small proofs (domain <= 2^prove_wide_log, default 2^21) run B, L and A on three auxiliary lanes of their
    own; large ones keep the two-lane layout (prover.hip groth16_sums_once).  Both layouts give the oracle's
    proof, for several witnesses in a row on the same context (the lanes' scratch arenas are reused)."""
    n_in, n_aux, rws, z = circuits.random_circuit(43, 5000)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rws, z)
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    op = oracle.OracleParams(oc, circuits.toxic())
    zb = circuits.z_bytes(z)
    want = [op.prove(zb, r, s)[0] for r, s in [(7, 8), (9, 10)]]
    for wide_log, b1_lane in (("0", "0"), ("21", "0"), ("21", "1"), ("21", "2")):
        tune.set("prove_wide_log", int(wide_log))
        tune.set("prove_b1_lane", int(b1_lane))
        got = [fg.prove(ctx, pk, gc, zb, r, s) for r, s in [(7, 8), (9, 10)]]
        assert got == want, f"prove_wide_log={wide_log} prove_b1_lane={b1_lane}"


def test_prove_rejects_mismatched_srs(ctx):
    n_in, n_aux, rws, z = circuits.random_circuit(51, 30)
    gc = fg.Circuit(ctx, len(rws), n_in, n_aux, circuits.to_csr(rws))
    n_in2, n_aux2, rws2, z2 = circuits.random_circuit(52, 200)
    gc2 = fg.Circuit(ctx, len(rws2), n_in2, n_aux2, circuits.to_csr(rws2))
    pk2 = fg.generate_random_parameters(ctx, gc2, circuits.toxic())
    with pytest.raises(fg.FilGpuError):
        fg.prove(ctx, pk2, gc, circuits.z_bytes(z), 1, 2)
    with pytest.raises(fg.FilGpuError):
        fg.prove(ctx, pk2, gc2, circuits.z_bytes(z2), fg.FR_MODULUS.to_bytes(32, "little"), 2)  # r >= r_mod


def test_groth16_trapdoor_2_20(ctx, oracle):
    """BASELINE-size property check: a 2^20-row synthetic circuit (GPU keygen from known toxic
    waste), checked by discrete logs: A == a*G1, B == b*G2, C == c*G1 where (a, b, c) follow
    from the QAP identity u(tau) v(tau) - w(tau) = h(tau) t(tau)."""
    import torch

    from fil_groth16 import synth

    sc = synth.SynthCircuit(log_rows=20, n_in=4, seed=9)
    gc = sc.load(ctx)
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    z = torch.from_numpy(np.frombuffer(sc.z_bytes(), dtype=np.uint8).copy()).cuda()
    r, s = circuits.blinding(3)
    proof, raw = fg.prove(ctx, pk, gc, z.data_ptr(), r, s, want_raw=True)
    a, b, c = fg.trapdoor_dlogs(ctx, pk, gc, z.data_ptr(), r, s)
    g1, g2 = oracle.g1_generator(), oracle.g2_generator()
    assert raw[:96] == oracle.g1_mul(g1, a)
    assert raw[96:288] == oracle.g2_mul(g2, b)
    assert raw[288:] == oracle.g1_mul(g1, c)
    vk, ic = pk.verifying_key()
    assert oracle.groth16_verify(vk, ic, sc.z_bytes()[:32 * sc.n_in], raw)


@pytest.mark.parametrize("name", ["random_11_24", "toy_chain_1022"])
def test_groth16_params_file_roundtrip(ctx, oracle, golden, name, tmp_path):
    """v28-style params files: a file written in bellman's layout from the oracle key loads through
    mi_params_load and proves the golden bytes; the GPU-generated key written by mi_params_write is
    byte-identical to it, and so is the verifying-key file."""
    import params_io

    g = golden["groth16"][name]
    n_in, n_aux, rows, z = _circuit_from_name(name)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rows, z)
    ex = oracle.OracleParams(oc, circuits.toxic()).export()
    ref = params_io.params_bytes(ex)
    p_ref = tmp_path / "oracle.params"
    p_ref.write_bytes(ref)
    pk = fg.ProvingKey.load_params(ctx, gc, str(p_ref), checked=True)
    r, s = circuits.blinding()
    assert fg.prove(ctx, pk, gc, circuits.z_bytes(z), r, s).hex() == g["proof"]
    gen = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    p_gen, p_vk = tmp_path / "gpu.params", tmp_path / "gpu.vk"
    gen.write_params(str(p_gen))
    gen.write_vk(str(p_vk))
    assert p_gen.read_bytes() == ref
    assert p_vk.read_bytes() == params_io.vk_bytes(ex)
    bad = tmp_path / "bad.params"
    bad.write_bytes(ref[:-1])
    with pytest.raises(fg.FilGpuError):
        fg.ProvingKey.load_params(ctx, gc, str(bad))


def test_seal_commit_phase2_self_verifies(ctx, oracle):
    """api/seal.hpp:296-313: partition proofs -> MultiProof -> batch self-verification; a partition
    with an unsatisfied witness makes the whole C2 call fail instead of returning a bad proof."""
    n_in, n_aux, rows, z = circuits.random_circuit(61, 500, n_in=5)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rows, z)
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    zb = circuits.z_bytes(z)
    blind = [(11 + k, 22 + k) for k in range(3)]
    buf = fg.seal_commit_phase2_proofs(ctx, pk, gc, [zb] * 3, blind, n_in)
    assert len(buf) == 3 * 192
    vk, ic = pk.verifying_key()
    for k in range(3):
        assert fg.verify(vk, ic, zb[32:32 * n_in], buf[192 * k:192 * (k + 1)])
    bad = bytearray(zb)
    bad[-32] ^= 1
    with pytest.raises(RuntimeError, match="sanity check failed"):
        fg.seal_commit_phase2_proofs(ctx, pk, gc, [zb, bytes(bad), zb], blind, n_in)


def test_window_and_winning_post_drivers(ctx, oracle):
    """api/post.hpp:305-348 / :178-230: the Window-PoSt driver proves one partition per
    get_partitions_for_window_post (sectors / 2349 per partition), on the high-priority stream, and
    each proof equals the oracle's; Winning-PoSt proves exactly one partition."""
    n_in, n_aux, rows, z = circuits.random_circuit(63, 400, n_in=4)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rows, z)
    tox = circuits.toxic()
    pk = fg.generate_random_parameters(ctx, gc, tox)
    op = oracle.OracleParams(oc, tox)
    zb = circuits.z_bytes(z)
    blind = [(31 + k, 41 + k) for k in range(3)]
    buf = fg.generate_window_post_proofs(ctx, pk, gc, 3 * 2349 + 7, 2349, [zb] * 3, blind)
    assert len(buf) == 3 * 192
    for k, (r, s) in enumerate(blind):
        assert buf[192 * k:192 * (k + 1)] == op.prove(zb, r, s)[0]
    with pytest.raises(ValueError, match="partition"):
        fg.generate_window_post_proofs(ctx, pk, gc, 3 * 2349, 2349, [zb] * 2, blind[:2])
    one = fg.generate_window_post_proofs(ctx, pk, gc, 2349, 2349, [zb], blind[:1])  # <= 1 -> one partition
    assert one == buf[:192]
    win = fg.generate_winning_post_proof(ctx, pk, gc, 1, 1, zb, blind[0])
    assert win == buf[:192]
    with pytest.raises(ValueError, match="invalid amount of replicas"):
        fg.generate_winning_post_proof(ctx, pk, gc, 2, 1, zb, blind[0])


@pytest.mark.parametrize("rows,seed,worlds", [(700, 81, (1, 2, 3, 7)), (16000, 82, (4,))])
def test_prove_share_vs_oracle_shares(ctx, oracle, rows, seed, worlds):
    """Single-proof latency mode: every rank's GPU share is byte-identical to the oracle's
    sums over the same slices, and the assembled proof equals the one-GPU proof and the oracle's."""
    import split_oracle

    n_in, n_aux, rws, z = circuits.random_circuit(seed, rows, n_in=6, n_free=32)
    mats = circuits.to_csr(rws)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rws, z)
    tox = circuits.toxic(seed)
    pk = fg.generate_random_parameters(ctx, gc, tox)
    op = oracle.OracleParams(oc, tox)
    zb = circuits.z_bytes(z)
    r, s = circuits.blinding(seed)
    vk, _ = pk.verifying_key()
    one = fg.prove(ctx, pk, gc, zb, r, s)
    assert one == op.prove(zb, r, s)[0]
    for world in worlds:
        shares = [fg.prove_share(ctx, pk, gc, zb, k, world) for k in range(world)]
        assert shares == split_oracle.shares(oracle, op, n_in, n_aux, mats, zb, world), world
        assert fg.assemble(vk, shares, r, s) == one, world
    with pytest.raises(fg.FilGpuError):
        fg.prove_share(ctx, pk, gc, zb, 2, 2)  # rank >= world


@pytest.mark.parametrize("rows,seed", [(700, 86), (16000, 87)])
def test_prove_share_ranges_vs_oracle(ctx, oracle, rows, seed):
    """Latency groups that compute H once (mi_groth16_prove_share_ranges, distributed.latency_ranges): every
    range share equals the oracle's sums over the same ranges, byte for byte, whether or not it holds H (only
    the shares with an H range run the witness map and NTT chain), and the shares of a partition assemble into
    the one-GPU proof.  Also an irregular partition (H split over two shares, empty ranges) and the device
    witness entry."""
    import torch

    import split_oracle
    from fil_groth16.distributed import latency_ranges

    n_in, n_aux, rws, z = circuits.random_circuit(seed, rows, n_in=6, n_free=32)
    mats = circuits.to_csr(rws)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rws, z)
    tox = circuits.toxic(seed)
    pk = fg.generate_random_parameters(ctx, gc, tox)
    op = oracle.OracleParams(oc, tox)
    zb = circuits.z_bytes(z)
    r, s = circuits.blinding(seed)
    vk, _ = pk.verifying_key()
    one = fg.prove(ctx, pk, gc, zb, r, s)
    sizes = (pk.n_h, pk.n_l, pk.n_a, pk.n_b)
    h, l, a, b = sizes
    parts = [latency_ranges(sizes, 3, 0.2), latency_ranges(sizes, 4, 0.0), latency_ranges(sizes, 2, 0.35),
             [[(0, h // 3), (0, 0), (0, a), (0, 0)], [(h // 3, h - h // 3), (0, l), (a, 0), (0, b // 2)],
              [(h, 0), (l, 0), (a, 0), (b // 2, b - b // 2)], [(0, 0), (0, 0), (0, 0), (0, 0)]]]
    zd = torch.from_numpy(np.frombuffer(zb, dtype=np.uint8).copy()).cuda()
    for i, rg in enumerate(parts):
        shares = [fg.prove_share_ranges(ctx, pk, gc, zd.data_ptr() if i % 2 else zb, x) for x in rg]
        assert shares == split_oracle.shares_ranges(oracle, op, n_in, n_aux, mats, zb, rg), i
        assert fg.assemble(vk, shares, r, s) == one, i
    with pytest.raises(fg.FilGpuError, match="range"):
        fg.prove_share_ranges(ctx, pk, gc, zb, [(1, h), (0, 0), (0, 0), (0, 0)])


def test_prove_share_device_witness(ctx, oracle):
    import torch

    n_in, n_aux, rws, z = circuits.random_circuit(83, 900, n_in=6, n_free=32)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rws, z)
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    zb = circuits.z_bytes(z)
    zd = torch.from_numpy(np.frombuffer(zb, dtype=np.uint8).copy()).cuda()
    vk, _ = pk.verifying_key()
    shares = [fg.prove_share(ctx, pk, gc, zd.data_ptr(), k, 3) for k in range(3)]
    assert fg.assemble(vk, shares, 9, 10) == fg.prove(ctx, pk, gc, zb, 9, 10)


def _split_gpu_worker(rank, world, port, outdir):
    import os
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "crypto3-fil-proofs_amd"), os.path.join(root, "tests", "golden")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import circuits
    import fil_groth16 as fg
    from fil_groth16.distributed import prove_split

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = fg.Context(0)
    n_in, n_aux, rws, z = circuits.random_circuit(84, 3000, n_in=6, n_free=32)
    gc = fg.Circuit(c, len(rws), n_in, n_aux, circuits.to_csr(rws))
    pk = fg.generate_random_parameters(c, gc, circuits.toxic())
    proof = prove_split(c, pk, gc, circuits.z_bytes(z), 21, 22, rank, world)
    with open(os.path.join(outdir, f"p{rank}.bin"), "wb") as f:
        f.write(proof)
    dist.barrier()
    dist.destroy_process_group()
    del pk, gc
    c.close()


def test_prove_split_two_processes(oracle, tmp_path):
    """fil_groth16.distributed.prove_split with one process per rank (both on this box's GPU, gloo for
    the 576-byte all-gather; RCCL on a multi-GPU node): every rank ends with the oracle's proof."""
    import socket

    import torch.multiprocessing as mp

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    mp.spawn(_split_gpu_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    outs = [open(tmp_path / f"p{k}.bin", "rb").read() for k in range(2)]
    n_in, n_aux, rws, z = circuits.random_circuit(84, 3000, n_in=6, n_free=32)
    op = oracle.OracleParams(oracle.OracleCircuit(len(rws), n_in, n_aux, circuits.to_csr(rws)), circuits.toxic())
    assert outs[0] == outs[1] == op.prove(circuits.z_bytes(z), 21, 22)[0]


def _balanced_gpu_worker(rank, world, port, outdir):
    import os
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "crypto3-fil-proofs_amd"), os.path.join(root, "tests", "golden")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import circuits
    import fil_groth16 as fg
    from fil_groth16.distributed import prove_partitions_balanced

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = fg.Context(0)
    n_in, n_aux, rws, z = circuits.random_circuit(85, 2500, n_in=5, n_free=32)
    gc = fg.Circuit(c, len(rws), n_in, n_aux, circuits.to_csr(rws))
    pk = fg.generate_random_parameters(c, gc, circuits.toxic())
    zb = circuits.z_bytes(z)
    vk, _ = pk.verifying_key()
    buf = prove_partitions_balanced(
        lambda ids: fg.prove_batch(c, pk, gc, [zb] * len(ids), [(31 + p, 41 + p) for p in ids]),
        lambda p, k, g: fg.prove_share(c, pk, gc, zb, k, g),
        lambda p, sh: fg.assemble(vk, sh, 31 + p, 41 + p), 3, rank, world)
    with open(os.path.join(outdir, f"b{rank}.bin"), "wb") as f:
        f.write(buf)
    dist.barrier()
    dist.destroy_process_group()
    del pk, gc
    c.close()


def test_balanced_partitions_two_processes(oracle, tmp_path):
    """The balanced config-5 runner on the GPU with one process per rank (both on this box's GPU, gloo for the
    all-gather): 3 partitions over 2 ranks -- 0 and 1 proven whole, 2 split into two latency-mode shares and
    assembled on both ranks -- give the oracle's serial multi-proof on every rank."""
    import socket

    import torch.multiprocessing as mp

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    mp.spawn(_balanced_gpu_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    outs = [open(tmp_path / f"b{k}.bin", "rb").read() for k in range(2)]
    n_in, n_aux, rws, z = circuits.random_circuit(85, 2500, n_in=5, n_free=32)
    op = oracle.OracleParams(oracle.OracleCircuit(len(rws), n_in, n_aux, circuits.to_csr(rws)), circuits.toxic())
    zb = circuits.z_bytes(z)
    assert outs[0] == outs[1] == b"".join(op.prove(zb, 31 + p, 41 + p)[0] for p in range(3))


def _srs_bcast_gpu_worker(rank, world, port, outdir):
    import os
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "crypto3-fil-proofs_amd"), os.path.join(root, "tests", "golden")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import circuits
    import fil_groth16 as fg
    from fil_groth16.distributed import broadcast_proving_key

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = fg.Context(0)
    n_in, n_aux, rws, z = circuits.random_circuit(85, 2000, n_in=4, n_free=16)
    gc = fg.Circuit(c, len(rws), n_in, n_aux, circuits.to_csr(rws))
    pk = fg.generate_random_parameters(c, gc, circuits.toxic()) if rank == 0 else None
    pk = broadcast_proving_key(c, pk, gc, rank, world, src=0, checked=True, chunk_bytes=1 << 16)
    proof = fg.prove(c, pk, gc, circuits.z_bytes(z), 31, 32)
    with open(os.path.join(outdir, f"b{rank}.bin"), "wb") as f:
        f.write(proof)
    dist.barrier()
    dist.destroy_process_group()
    del pk, gc
    c.close()


def test_srs_broadcast_two_processes(oracle, tmp_path):
    """fil_groth16.distributed.broadcast_proving_key: rank 0 holds the key, rank 1 receives it over the
    process group (checked load: subgroup checks on every point) and proves; both equal the oracle proof."""
    import socket

    import torch.multiprocessing as mp

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    mp.spawn(_srs_bcast_gpu_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    outs = [open(tmp_path / f"b{k}.bin", "rb").read() for k in range(2)]
    n_in, n_aux, rws, z = circuits.random_circuit(85, 2000, n_in=4, n_free=16)
    op = oracle.OracleParams(oracle.OracleCircuit(len(rws), n_in, n_aux, circuits.to_csr(rws)), circuits.toxic())
    assert outs[0] == outs[1] == op.prove(circuits.z_bytes(z), 31, 32)[0]


def test_production_random_blinding_entries(ctx, oracle):
    """crypto3 prove / bellman create_random_proof: r, s drawn inside the library (getrandom).  The proofs
    verify, differ between calls on the same witness, and the batch-routed compound.circuit_proofs with
    injected (r, s) still equals the oracle proof for proof."""
    n_in, n_aux, rows, z = circuits.random_circuit(65, 300, n_in=4)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rows, z)
    tox = circuits.toxic()
    pk = fg.generate_random_parameters(ctx, gc, tox)
    op = oracle.OracleParams(oc, tox)
    zb = circuits.z_bytes(z)
    vk, ic = pk.verifying_key()
    p1, p2 = fg.prove(ctx, pk, gc, zb), fg.prove(ctx, pk, gc, zb)
    assert p1 != p2
    assert fg.verify(vk, ic, zb[32:32 * n_in], p1) and fg.verify(vk, ic, zb[32:32 * n_in], p2)
    import torch

    zd = torch.from_numpy(np.frombuffer(zb, dtype=np.uint8).copy()).cuda()
    assert fg.verify(vk, ic, zb[32:32 * n_in], fg.prove(ctx, pk, gc, zd.data_ptr()))
    rand = fg.circuit_proofs(ctx, pk, gc, [zb] * 3)
    assert len(set(rand)) == 3 and all(fg.verify(vk, ic, zb[32:32 * n_in], p) for p in rand)
    blind = [(7 + k, 9 + k) for k in range(3)]
    assert fg.circuit_proofs(ctx, pk, gc, [zb] * 3, blind) == [op.prove(zb, r, s)[0] for r, s in blind]
    buf = fg.seal_commit_phase2_proofs(ctx, pk, gc, [zb] * 2)
    assert all(fg.verify(vk, ic, zb[32:32 * n_in], buf[192 * k:192 * k + 192]) for k in range(2))


def test_get_groth_params_read_or_generate(ctx, oracle, golden, tmp_path, monkeypatch):
    """get_groth_params / get_verifying_key (core/parameter_cache.hpp:185-219) through mi_get_groth_params: the
    first call finds no v28-<id>.params under FIL_PROOFS_PARAMETER_CACHE, generates the key and writes the params
    and vk files (byte-identical to the oracle key's bellman layout); the second call loads the file instead and
    proves the golden bytes; a corrupt file is regenerated, as the reference's catch-all does."""
    import params_io

    monkeypatch.setenv("FIL_PROOFS_PARAMETER_CACHE", str(tmp_path))
    g = golden["groth16"]["random_11_24"]
    n_in, n_aux, rows, z = _circuit_from_name("random_11_24")
    oc, gc = _load(ctx, oracle, n_in, n_aux, rows, z)
    ex = oracle.OracleParams(oc, circuits.toxic()).export()
    cid = fg.param_cache_id("test-circuit", "random_11_24{n_in: %d, n_aux: %d}" % (n_in, n_aux))
    r, s = circuits.blinding()
    pk1, gen1 = fg.get_groth_params(ctx, gc, cid, toxic=circuits.toxic())
    assert gen1
    assert (tmp_path / f"v28-{cid}.params").read_bytes() == params_io.params_bytes(ex)
    assert (tmp_path / f"v28-{cid}.vk").read_bytes() == params_io.vk_bytes(ex)
    pk2, gen2 = fg.get_groth_params(ctx, gc, cid, toxic=[1, 2, 3, 4, 5])  # toxic unused: the file is read
    assert not gen2
    assert fg.prove(ctx, pk1, gc, circuits.z_bytes(z), r, s).hex() == g["proof"]
    assert fg.prove(ctx, pk2, gc, circuits.z_bytes(z), r, s).hex() == g["proof"]
    p = tmp_path / f"v28-{cid}.params"
    p.write_bytes(p.read_bytes()[:-5])
    pk3, gen3 = fg.get_groth_params(ctx, gc, cid)  # corrupt -> regenerated from OS randomness, valid proof
    assert gen3 and fg.params_inspect(str(p))["h"] == len(ex["h"]) // 96
    # the stale .vk of the first parameters is replaced by the regenerated key's own
    pk3.write_vk(str(tmp_path / "pk3.vk"))
    assert (tmp_path / f"v28-{cid}.vk").read_bytes() == (tmp_path / "pk3.vk").read_bytes() != params_io.vk_bytes(ex)
    vk, ic = pk3.verifying_key()
    raw = fg.prove(ctx, pk3, gc, circuits.z_bytes(z), r, s, want_raw=True)[1]
    assert oracle.groth16_verify(vk, ic, circuits.z_bytes(z)[:32 * n_in], raw)


@pytest.mark.parametrize("rows,seed", [(700, 91), (5000, 92)])
def test_h_split_shares_vs_oracle(ctx, oracle, rows, seed):
    """H computed once and split (mi_groth16_h_coeffs_dev + mi_groth16_prove_share_ranges_h_dev): the exported H
    coefficients equal the oracle's in the device's bit-reversed order; H-only, L/A/B-only and mixed shares from the
    received coefficients equal the oracle's range sums byte for byte; the shares of hsplit_shares over 2-4 ranks
    assemble into the one-GPU proof; non-canonical coefficients are refused."""
    import torch

    import split_oracle
    from fil_groth16.distributed import hsplit_fractions, hsplit_shares, latency_ranges_hsplit

    n_in, n_aux, rws, z = circuits.random_circuit(seed, rows, n_in=6, n_free=32)
    mats = circuits.to_csr(rws)
    oc, gc = _load(ctx, oracle, n_in, n_aux, rws, z)
    tox = circuits.toxic(seed)
    pk = fg.generate_random_parameters(ctx, gc, tox)
    op = oracle.OracleParams(oc, tox)
    zb = circuits.z_bytes(z)
    r, s = circuits.blinding(seed)
    vk, _ = pk.verifying_key()
    one = fg.prove(ctx, pk, gc, zb, r, s)
    zd = torch.from_numpy(np.frombuffer(zb, dtype=np.uint8).copy()).cuda()
    hbuf = torch.zeros(32 * gc.d, dtype=torch.uint8, device="cuda")
    fg.h_coeffs_dev(ctx, gc, zd.data_ptr(), hbuf.data_ptr())
    want_h = split_oracle.h_coeffs_perm(op, zb)
    assert hbuf.cpu().numpy().tobytes() == want_h
    sizes = (pk.n_h, pk.n_l, pk.n_a, pk.n_b)
    h, l, a, b = sizes
    rg = [[(0, h // 3), (0, 0), (0, 0), (0, 0)], [(h // 3, h - h // 3), (0, l // 2), (0, a), (0, 0)],
          [(0, 0), (l // 2, l - l // 2), (a, 0), (0, b)]]
    got = [fg.prove_share_ranges(ctx, pk, gc, zd.data_ptr(), x, h_dev=hbuf.data_ptr()) for x in rg]
    assert got == split_oracle.shares_ranges(oracle, op, n_in, n_aux, mats, zb, rg)
    assert fg.assemble(vk, got, r, s) == one
    for g in (2, 3, 4):
        hl, fl = hsplit_fractions(10.0, 20.0, 50.0, g)
        ranges = latency_ranges_hsplit(sizes, g, hl, fl)
        hbuf.zero_()
        shs = []
        for k in range(g):  # rank 0 first, as the group runs it (its coefficients stay in hbuf)

            def h_coeffs(*arg):
                if not arg:
                    fg.h_coeffs_dev(ctx, gc, zd.data_ptr(), hbuf.data_ptr())
                return hbuf

            shs += hsplit_shares(k, ranges, h_coeffs,
                                 lambda x, hh: fg.prove_share_ranges(ctx, pk, gc, zd.data_ptr(), x,
                                                                     h_dev=hh.data_ptr() if hh is not None else None),
                                 lambda t: (lambda: t))
        assert len(shs) == 2 * g - 1
        assert fg.assemble(vk, shs, r, s) == one, g
    bad = hbuf.clone()
    bad[32 * 5:32 * 6] = 0xFF  # coefficient 5 >= r
    with pytest.raises(fg.FilGpuError) as e:
        fg.prove_share_ranges(ctx, pk, gc, zd.data_ptr(), rg[0], h_dev=bad.data_ptr())
    assert e.value.code == -1
