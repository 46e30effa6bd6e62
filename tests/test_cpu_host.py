"""CPU: the C-ABI library loads and exports every declared symbol; host-side logic mirrors the
reference (partition counts, multi-proof layout, sharding); the synthetic workload generator is
satisfiable (checked by the oracle).  No GPU compute is called here."""
import ctypes
import os
import re

import pytest

import circuits
import fil_groth16 as fg
from fil_groth16 import compound, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    names = set()
    inc = os.path.join(ROOT, "include")
    for fn in os.listdir(inc):
        if fn.endswith(".h"):
            src = open(os.path.join(inc, fn)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            names |= set(re.findall(r"\b(mi_\w+)\s*\(", src))
    return names


def test_library_exports_every_declared_symbol():
    L = fg.lib()
    declared = _declared_functions()
    assert len(declared) >= 35
    assert declared == set(fg.EXPORTS), declared ^ set(fg.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name


def test_library_is_gfx950_code_object():
    data = open(fg.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"k_accum_level0" in data and b"k_ntt_pass" in data


def test_window_heuristic():
    assert fg.msm_window_bits(1 << 20) == 16
    assert 18 <= fg.msm_window_bits(1 << 26) <= 22
    assert fg.msm_window_bits(1) >= 4


def test_partition_count_semantics():
    # core/partitions.hpp:36-38
    assert compound.partition_count(-1) == 1
    assert compound.partition_count(0) == -1
    assert compound.partition_count(10) == 10


def test_window_post_partitions():
    # libs/filecoin/src/api/post.cpp:37-46 (integer quotient; None when <= 1)
    assert compound.get_partitions_for_window_post(2349, 2349) is None
    assert compound.get_partitions_for_window_post(2349 * 10, 2349) == 10
    assert compound.get_partitions_for_window_post(2349 * 10 + 5, 2349) == 10
    assert compound.get_partitions_for_window_post(1, 2) is None


def test_multiproof_layout():
    proofs = [bytes([i]) * 192 for i in range(10)]
    mp = fg.MultiProof(proofs, verifying_key=b"vk")
    buf = mp.to_bytes()
    assert len(buf) == 1920  # 10 partitions x SINGLE_PARTITION_PROOF_LEN (constants.hpp:93)
    assert fg.MultiProof.from_bytes(buf).circuit_proofs == proofs
    with pytest.raises(ValueError):
        fg.MultiProof.from_bytes(buf[:-1])
    with pytest.raises(ValueError):
        compound.circuit_proofs(None, None, None, [], [])


def test_shard_partitions_round_robin():
    # config 5: 10 partitions on 8 GPUs -> ranks 0, 1 prove two
    shards = [compound.shard_partitions(10, r, 8) for r in range(8)]
    assert shards[0] == [0, 8] and shards[1] == [1, 9] and shards[7] == [7]
    assert sorted(p for s in shards for p in s) == list(range(10))


def test_fr_bytes():
    assert fg.fr_bytes(fg.FR_MODULUS + 3) == (3).to_bytes(32, "little")
    raw = fg.FR_MODULUS.to_bytes(32, "little")
    assert fg.fr_bytes(raw) == raw


@pytest.mark.parametrize("log_rows,n_in", [(6, 1), (10, 4), (14, 7)])
def test_synthetic_circuit_satisfied(oracle, log_rows, n_in):
    sc = synth.SynthCircuit(log_rows, n_in, seed=3)
    assert sc.n + sc.n_in == 1 << log_rows
    oc = oracle.OracleCircuit(sc.n, sc.n_in, sc.n_aux, sc.csr())
    z = sc.z_bytes()
    assert oc.satisfied(z)
    bad = bytearray(z)
    bad[-32] ^= 1
    assert not oc.satisfied(bytes(bad))


@pytest.mark.parametrize("log_rows,n_in", [(6, 1), (12, 4)])
def test_synthetic_uniform_witness(oracle, log_rows, n_in):
    """MI_SYNTH_UNIFORM_WITNESS: the same row shapes without boolean rows -- satisfied, same domain, and almost
    no small aux values (the boolean-heavy default has a quarter of them in {0, 1})."""
    sc = synth.SynthCircuit(log_rows, n_in, seed=3, uniform=True)
    assert sc.n + sc.n_in == 1 << log_rows
    oc = oracle.OracleCircuit(sc.n, sc.n_in, sc.n_aux, sc.csr())
    assert oc.satisfied(sc.z_bytes())
    aux = sc.z_array().reshape(-1, 32)[n_in:]
    small = int((aux[:, 4:] == 0).all(axis=1).sum())  # values below 2^32
    mixed = synth.SynthCircuit(log_rows, n_in, seed=3).z_array().reshape(-1, 32)[n_in:]
    assert small <= len(aux) // 64 < int((mixed[:, 4:] == 0).all(axis=1).sum())


def test_synthetic_circuit_deterministic():
    a = synth.SynthCircuit(12, 4, seed=5).z_bytes()
    b = synth.SynthCircuit(12, 4, seed=5).z_bytes()
    c = synth.SynthCircuit(12, 4, seed=6).z_bytes()
    assert a == b and a != c


def test_synthetic_small_groth16_oracle(oracle):
    """The oracle proves the synthetic circuit and the pairing verifier accepts it (end-to-end CPU
    check of the workload family the bench times)."""
    sc = synth.SynthCircuit(9, 4, seed=2)
    oc = oracle.OracleCircuit(sc.n, sc.n_in, sc.n_aux, sc.csr())
    P = oracle.OracleParams(oc, circuits.toxic())
    z = sc.z_bytes()
    proof, raw, _ = P.prove(z, 11, 12)
    ex = P.export()
    assert oracle.groth16_verify(ex["vk"], ex["ic"], z[:32 * sc.n_in], raw)


def test_no_gpu_raises_loudly():
    """Without a GPU the compute path fails loudly (no CPU fallback)."""
    n = ctypes.c_int(-1)
    fg.lib().mi_device_count(ctypes.byref(n))
    if n.value > 0:
        pytest.skip("GPU present")
    with pytest.raises(fg.FilGpuError):
        fg.Context(0)


def test_cpp_host_layer_builds_and_fails_loudly_without_gpu():
    """include/mi355x_groth16.hpp compiles against the C ABI; without a device the example exits
    with MI_ERR_NO_DEVICE (3) instead of computing anything on the CPU."""
    import subprocess

    pkg = os.path.join(ROOT, "crypto3-fil-proofs_amd")
    subprocess.check_call(["make", "-s", "-C", pkg, "build/prove_synthetic"])
    exe = os.path.join(pkg, "build", "prove_synthetic")
    n = ctypes.c_int(-1)
    fg.lib().mi_device_count(ctypes.byref(n))
    if n.value > 0:
        pytest.skip("GPU present (covered by tests/test_gpu_cpp.py)")
    r = subprocess.run([exe, "8", "2"], capture_output=True, text=True)
    assert r.returncode == 3 and "no HIP device" in r.stderr


def test_post_partition_derivation():
    # generate_window_post: get_partitions_for_window_post's optional -> FallbackPoStCompound partitions
    # (unset = partition_count(-1) = 1); api/post.hpp:319-322, src/api/post.cpp:37-46
    from fil_groth16.compound import _post_partitions
    assert _post_partitions(10 * 2349, 2349) == 10
    assert _post_partitions(10 * 2349 + 2348, 2349) == 10
    assert _post_partitions(2349, 2349) == 1
    assert _post_partitions(5, 2349) == 1


def test_tuning_switches_are_explicit_not_environment():
    """the library reads no environment variable that changes window sizes, lanes, kernels or hash
    constants; the A/B switches are set through mi_tune_set (test only), and an unknown name is refused.  The only
    getenv left in csrc/ is FIL_PROOFS_PARAMETER_CACHE (the reference's parameter-cache directory,
    parameter_cache.hpp:52)."""
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "crypto3-fil-proofs_amd", "csrc")
    reads = []
    for f in sorted(os.listdir(csrc)):
        with open(os.path.join(csrc, f)) as fh:
            reads += re.findall(r'getenv\("([A-Z0-9_]+)"\)', fh.read())
    assert reads == ["FIL_PROOFS_PARAMETER_CACHE"], reads
    assert fg.tune_get("msm_c") is None
    with fg.tuned(msm_c=12, prove_lanes=1):
        assert fg.tune_get("msm_c") == 12 and fg.tune_get("prove_lanes") == 1
        assert fg.msm_window_bits(1 << 20) == 12  # the window heuristic follows the switch
    assert fg.tune_get("msm_c") is None and fg.tune_get("prove_lanes") is None
    with pytest.raises(fg.FilGpuError):
        fg.tune_set("no_such_switch", 1)
    os.environ["MI_MSM_C"] = "9"  # the old environment knob no longer changes anything
    try:
        assert fg.msm_window_bits(1 << 20) != 9
    finally:
        del os.environ["MI_MSM_C"]


def test_select_challenges_reference_vectors():
    """libs/filecoin/test/parameters.cpp:35-43 (partition_layer_challenges_test): select_challenges(p, 12, 11)
    .challenges_count_all() is 12 / 6 / 3 for 1 / 2 / 4 partitions (and 6 for PoRepProofPartitions(2)); the
    function is proofs/parameters.hpp:90-99.  The 32 / 64 GiB PoRep partitions take 11 layers x 18 challenges
    (176 minimum over 10 partitions, constants.hpp:65-78); the small sizes 2 x 2."""
    f = lambda p: compound.select_challenges(p, 12, 11).challenges_count_all()  # noqa: E731
    assert (f(1), f(2), f(4)) == (12, 6, 3)
    assert compound.select_challenges(2, 12, 11).layers == 11
    assert compound.porep_layer_challenges(compound.SECTOR_SIZE_32GIB) == (11, 18)
    assert compound.porep_layer_challenges(compound.SECTOR_SIZE_64GIB) == (11, 18)
    assert compound.porep_layer_challenges(2048) == (2, 2)
    assert compound.select_challenges(3, 10, 2).challenges_count_all() == 4  # the smallest count reaching 10
    with pytest.raises(ValueError):
        compound.select_challenges(0, 12, 11)
