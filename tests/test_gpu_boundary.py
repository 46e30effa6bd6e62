"""GPU: input validation and the host-witness paths of the C ABI.

* Non-canonical witness entries (>= r) are refused with MI_ERR_ARG on every prove entry point, host
  and device witnesses alike: an Fr32 "MUST represent a valid Fr" (core/fr32.hpp:36-40), and the
  reference's own tripwire feeds all-0xFF bytes (libs/filecoin/test/api/mod.cpp:35-44).
* prove_batch with witnesses in pinned (mi_host_alloc), numpy and bytes memory, the upload of
  partition k + 1 overlapping proof k: every proof equals the oracle's.
* Proving keys are read with bellman's Parameters::read rules: flag bits, the identity refused in every
  query and in ic, curve membership, and r P == O when checked (points on the curve outside the
  prime-order subgroup load unchecked and are refused checked).
"""
import numpy as np
import pytest

import badpoints
import circuits
import fil_groth16 as fg
from pyref import R

pytestmark = pytest.mark.gpu

MI_ERR_ARG = -1


@pytest.fixture(scope="module")
def case(ctx, oracle):
    n_in, n_aux, rows, z = circuits.random_circuit(71, 400, n_in=5)
    mats = circuits.to_csr(rows)
    gc = fg.Circuit(ctx, len(rows), n_in, n_aux, mats)
    pk = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    op = oracle.OracleParams(oracle.OracleCircuit(len(rows), n_in, n_aux, mats), circuits.toxic())
    return {"gc": gc, "pk": pk, "op": op, "z": z, "n_in": n_in, "mats": mats, "rows": rows, "n_aux": n_aux}


def _with(z, index, value):
    zb = bytearray(circuits.z_bytes(z))
    zb[32 * index:32 * index + 32] = value.to_bytes(32, "little")
    return bytes(zb)


def _dev(b):
    import torch

    return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).cuda()


@pytest.mark.parametrize("value", [R, R + 5, 2**256 - 1])
def test_witness_non_canonical_refused(ctx, case, value):
    gc, pk, z = case["gc"], case["pk"], case["z"]
    good = circuits.z_bytes(z)
    for index in (1, len(z) - 1):
        bad = _with(z, index, value)
        with pytest.raises(fg.FilGpuError, match="canonical") as e:
            fg.prove(ctx, pk, gc, bad, 1, 2)
        assert e.value.code == MI_ERR_ARG
        bd = _dev(bad)
        with pytest.raises(fg.FilGpuError, match="canonical"):
            fg.prove(ctx, pk, gc, bd.data_ptr(), 1, 2)
        with pytest.raises(fg.FilGpuError, match="canonical"):
            fg.prove_batch(ctx, pk, gc, [good, bad, good], [(1, 2), (3, 4), (5, 6)])
        with pytest.raises(fg.FilGpuError, match="canonical"):
            fg.prove_share(ctx, pk, gc, bad, 0, 2)
        with pytest.raises(fg.FilGpuError, match="canonical"):
            fg.prove_share(ctx, pk, gc, bd.data_ptr(), 1, 2)
    # the context is still usable and exact after the refusals
    assert fg.prove(ctx, pk, gc, good, 1, 2) == case["op"].prove(good, 1, 2)[0]


def test_prove_batch_host_witness_kinds(ctx, case):
    """Four partitions (distinct witnesses: z with its last entry shifted, unsatisfied but canonical; the
    prover is a deterministic map either way) from pinned, numpy and bytes memory."""
    gc, pk, z, op = case["gc"], case["pk"], case["z"], case["op"]
    ws = [_with(z, len(z) - 1, (z[-1] + k) % R) for k in range(4)]
    hb0, hb3 = fg.HostBuffer(len(ws[0])), fg.HostBuffer(len(ws[3]))
    hb0.array[:] = np.frombuffer(ws[0], dtype=np.uint8)
    hb3.array[:] = np.frombuffer(ws[3], dtype=np.uint8)
    rs = [(10 + k, 20 + k) for k in range(4)]
    ctx.reset_stats()
    proofs = fg.prove_batch(ctx, pk, gc, [hb0, np.frombuffer(ws[1], dtype=np.uint8), ws[2], hb3], rs)
    for k in range(4):
        assert proofs[k] == op.prove(ws[k], *rs[k])[0], k
    st = ctx.stats()
    assert st["h2d"]["launches"] == 4 and st["h2d"]["units"] == 4 * len(ws[0])
    assert st["prove"]["launches"] == 4


def _export(oracle):
    n_in, n_aux, rows, z = circuits.random_circuit(11, 24)
    mats = circuits.to_csr(rows)
    oc = oracle.OracleCircuit(len(rows), n_in, n_aux, mats)
    return n_in, n_aux, rows, z, mats, oracle.OracleParams(oc, circuits.toxic()).export()


def _load(ctx, gc, ex, checked, **repl):
    q = {k: bytearray(ex[k]) for k in ("vk", "ic", "h", "l", "a", "b_g1", "b_g2")}
    for key, (off, data) in repl.items():
        q[key][off:off + len(data)] = data
    return fg.ProvingKey.load(ctx, gc, *(bytes(q[k]) for k in ("vk", "ic", "h", "l", "a", "b_g1", "b_g2")),
                              checked=checked)


def test_srs_subgroup_checked_vs_unchecked(ctx, oracle):
    n_in, n_aux, rows, z, mats, ex = _export(oracle)
    gc = fg.Circuit(ctx, len(rows), n_in, n_aux, mats)
    _, p1 = badpoints.g1_non_subgroup()
    _, p2 = badpoints.g2_non_subgroup()
    for key, off, data in (("l", 96, p1), ("h", 0, p1), ("b_g2", 192, p2), ("b_g1", 0, p1)):
        _load(ctx, gc, ex, False, **{key: (off, data)})  # on the curve: the unchecked read accepts it
        with pytest.raises(fg.FilGpuError, match="subgroup") as e:
            _load(ctx, gc, ex, True, **{key: (off, data)})
        assert e.value.code == MI_ERR_ARG
    with pytest.raises(fg.FilGpuError, match="subgroup"):
        _load(ctx, gc, ex, True, vk=(0, p1))  # alpha_g1
    with pytest.raises(fg.FilGpuError, match="subgroup"):
        _load(ctx, gc, ex, True, ic=(96, p1))
    # the untouched key loads checked and proves the golden bytes
    pk = _load(ctx, gc, ex, True)
    r, s = circuits.blinding()
    assert fg.prove(ctx, pk, gc, circuits.z_bytes(z), r, s) == oracle.OracleParams(
        oracle.OracleCircuit(len(rows), n_in, n_aux, mats), circuits.toxic()).prove(circuits.z_bytes(z), r, s)[0]


INF_G1 = bytes([0x40]) + bytes(95)


@pytest.mark.parametrize("checked", [False, True])
def test_srs_refuses_infinity_and_bad_flags(ctx, oracle, checked):
    n_in, n_aux, rows, z, mats, ex = _export(oracle)
    gc = fg.Circuit(ctx, len(rows), n_in, n_aux, mats)
    for key, off, data in (("h", 0, INF_G1), ("l", 96, INF_G1), ("a", 0, INF_G1),
                           ("b_g2", 0, bytes([0x40]) + bytes(191)), ("ic", 0, INF_G1)):
        with pytest.raises(fg.FilGpuError, match="infinity"):
            _load(ctx, gc, ex, checked, **{key: (off, data)})
    h0 = ex["h"][:96]
    for bad in (bytes([h0[0] | 0x80]) + h0[1:],           # compression flag on an uncompressed point
                bytes([h0[0] | 0x20]) + h0[1:],           # sort flag on a finite point
                bytes([0x40]) + bytes(94) + b"\x01",      # infinity with a non-zero payload
                bytes([0x60]) + bytes(95)):               # infinity with the sort flag
        with pytest.raises(fg.FilGpuError, match="malformed"):
            _load(ctx, gc, ex, checked, h=(0, bad))
    off_curve = bytearray(ex["vk"][:96])
    off_curve[95] ^= 1
    with pytest.raises(fg.FilGpuError, match="curve"):
        _load(ctx, gc, ex, checked, vk=(0, bytes(off_curve)))
    with pytest.raises(fg.FilGpuError):
        _load(ctx, gc, ex, checked, vk=(0, bytes([0xA0]) + bytes(95)))  # flags on the vk too


def test_msm_bases_flag_rules(ctx, oracle):
    """MSM bases (mi_msm_g1 / mi_points_upload_g1) accept the identity but not malformed flags."""
    n_in, n_aux, rows, z, mats, ex = _export(oracle)
    b = ex["h"][:96 * 4]
    sc = (5).to_bytes(32, "little") * 4
    assert ctx.msm_g1(INF_G1 + b[96:], sc) == oracle.msm_g1(INF_G1 + b[96:], sc)
    with pytest.raises(fg.FilGpuError):
        ctx.msm_g1(bytes([b[0] | 0x80]) + b[1:], sc)


def test_srs_stream_load_chunks_host_and_device(ctx, oracle):
    """mi_srs_stream_*: the key arrives in chunks (the receiving side of broadcast_proving_key), from host
    memory and from device memory, and proves the oracle's bytes; a chunk out of order, a missing tail and a
    non-subgroup point under checked are refused.  Source chunks come from mi_srs_export_query_dev."""
    import torch

    n_in, n_aux, rows, z, mats, ex = _export(oracle)
    gc = fg.Circuit(ctx, len(rows), n_in, n_aux, mats)
    pk0 = fg.generate_random_parameters(ctx, gc, circuits.toxic())
    counts = [pk0.n_h, pk0.n_l, pk0.n_a, pk0.n_b, pk0.n_b]
    vk, ic = pk0.verifying_key()
    r, s = circuits.blinding()
    want = oracle.OracleParams(oracle.OracleCircuit(len(rows), n_in, n_aux, mats), circuits.toxic()).prove(
        circuits.z_bytes(z), r, s)[0]
    for on_device in (False, True):
        st = fg.ProvingKey.stream_begin(ctx, gc, vk, ic, counts, checked=True)
        for q in range(5):
            esz = 192 if q == 4 else 96
            for first in range(0, counts[q], 7):
                m = min(7, counts[q] - first)
                t = torch.empty(esz * m, dtype=torch.uint8, device="cuda")
                pk0.export_query_dev(q, first, m, t.data_ptr())
                assert t.cpu().numpy().tobytes() == pk0.query(q)[esz * first:esz * (first + m)]
                if on_device:
                    st.part(q, first, t.data_ptr(), m, on_device=True)
                else:
                    st.part(q, first, t.cpu().numpy(), m)
        pk = st.end()
        assert fg.prove(ctx, pk, gc, circuits.z_bytes(z), r, s) == want
    st = fg.ProvingKey.stream_begin(ctx, gc, vk, ic, counts)
    with pytest.raises(fg.FilGpuError, match="order"):
        st.part(0, 1, ex["h"][96:192], 1)
    st.part(0, 0, ex["h"][:96], 1)
    with pytest.raises(fg.FilGpuError, match="incomplete"):
        st.end()
    _, bad = badpoints.g1_non_subgroup()
    st = fg.ProvingKey.stream_begin(ctx, gc, vk, ic, counts, checked=True)
    for q, name in enumerate(("h", "l", "a", "b_g1", "b_g2")):
        data = bytearray(pk0.query(q))
        if name == "l":
            data[:96] = bad
        st.part(q, 0, bytes(data), counts[q])
    with pytest.raises(fg.FilGpuError, match="subgroup"):
        st.end()


# The reference's Fr32 canonicality edge (libs/storage/test/core/fr32.cpp:51-86, bytes_into_fr accept /
# refuse) and the api tripwire (libs/filecoin/test/api/mod.cpp:35-44: all-zero converts, all-0xFF does not),
# as 32-byte little-endian encodings with the reference's expected verdict.
FR32_VECTORS = [
    ("fr32.cpp:52 bytes 0..31", bytes(range(32)), True),
    ("fr32.cpp:58 ff..ff,115", b"\xff" * 31 + bytes([115]), False),
    ("fr32.cpp:65 ff..ff,114", b"\xff" * 31 + bytes([114]), True),
    ("fr32.cpp:72 ff..ff,236,115", b"\xff" * 30 + bytes([236, 115]), True),
    ("fr32.cpp:79 ff..ff,237,115", b"\xff" * 30 + bytes([237, 115]), False),
    ("mod.cpp:36 all zero", bytes(32), True),
    ("mod.cpp:41 all 0xff", b"\xff" * 32, False),
]


@pytest.mark.parametrize("name,enc,ok", FR32_VECTORS, ids=[v[0] for v in FR32_VECTORS])
def test_fr32_reference_vectors_through_the_c_abi(ctx, case, name, enc, ok):
    """Each vector as a witness entry (host and device witness, prove_batch, prove_share) and as an instance
    slot of the library-built PoSt circuit (mi_stacked_public_inputs, mi_stacked_witness, _dev): accepted
    exactly when the reference accepts it, refused with MI_ERR_ARG ("canonical") otherwise."""
    from fil_groth16 import stacked

    assert (int.from_bytes(enc, "little") < R) == ok
    gc, pk, z = case["gc"], case["pk"], case["z"]
    good = circuits.z_bytes(z)
    zb = bytearray(good)
    zb[32:64] = enc  # input 1
    zb = bytes(zb)
    calls = [lambda: fg.prove(ctx, pk, gc, zb, 1, 2),
             lambda: fg.prove(ctx, pk, gc, _dev(zb).data_ptr(), 1, 2),
             lambda: fg.prove_batch(ctx, pk, gc, [good, zb], [(1, 2), (3, 4)]),
             lambda: fg.prove_share(ctx, pk, gc, zb, 0, 2),
             lambda: fg.prove_share(ctx, pk, gc, _dev(zb).data_ptr(), 1, 2)]
    pc = stacked.FallbackPoStCircuit(1, 1, 64, 8, 0, 0, with_r1cs=False)
    import stacked_instance as si

    slots = bytearray(stacked.post_slots(pc, si.generate_post(1, 1, 64, (8, 0, 0), seed=2)["sectors"]))
    slots[32 * 1:32 * 2] = enc  # comm_c of the sector (a free field element of the instance)
    slots = bytes(slots)
    zdev = _dev(bytes(32 * pc.num_vars))
    calls += [lambda: pc.public_inputs(slots), lambda: pc.witness(ctx, slots),
              lambda: pc.witness_dev(ctx, _dev(slots).data_ptr(), zdev.data_ptr())]
    for i, call in enumerate(calls):
        if ok:
            call()
        else:
            with pytest.raises(fg.FilGpuError, match="canonical") as e:
                call()
            assert e.value.code == MI_ERR_ARG, i
    assert fg.prove(ctx, pk, gc, good, 1, 2) == case["op"].prove(good, 1, 2)[0]
