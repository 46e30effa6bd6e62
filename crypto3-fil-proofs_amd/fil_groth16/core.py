"""Python mirror of the prover-side reference interface, over the C ABI.

Reference names kept (paths relative to the reference root):
  * ``Context``      one per GPU -- the device-side counterpart of the process-wide Groth param
                     cache (libs/filecoin/include/nil/filecoin/proofs/caches.hpp:48-67)
  * ``Circuit``      the R1CS a compound proof synthesises (e.g. StackedCompound::circuit,
                     libs/storage/.../porep/stacked/circuit/proof.hpp:271-299)
  * ``ProvingKey``   r1cs_gg_ppzksnark_mapped_scheme_params / scheme_params{vk,h,l,a,b_g1,b_g2}
                     (core/crypto/scheme_params.hpp:38-67, core/crypto/mapped_scheme_params.hpp:43-84)
  * ``prove``        crypto3 r1cs_gg_ppzksnark prove(pk, primary_input, auxiliary_input) -> proof
                     (called from compound_proof::circuit_proofs, core/proof/compound_proof.hpp:127-137)
  * ``generate_random_parameters``   groth16::generate_random_parameters (core/parameter_cache.hpp:190)
Errors raise ``FilGpuError`` (the reference asserts / throws: compound_proof.hpp:94).
"""
import ctypes
import os

import numpy as np

from ._lib import check, lib, torch_sync

FR_MODULUS = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
PROOF_BYTES = 192
SHARE_BYTES = 576
VK_BYTES = 864


def fr_bytes(x) -> bytes:
    """int -> 32-byte LE canonical; 32-byte values pass through unchanged (the library rejects
    non-canonical blinding values rather than reducing them)."""
    if isinstance(x, (bytes, bytearray)):
        assert len(x) == 32
        return bytes(x)
    return int(x % FR_MODULUS).to_bytes(32, "little")


def _ptr(b):
    """(ctypes pointer, keepalive) for bytes / bytearray / numpy buffers."""
    if isinstance(b, np.ndarray):
        assert b.flags.c_contiguous
        return ctypes.c_void_p(b.ctypes.data), b
    if isinstance(b, (bytes, bytearray, memoryview)):
        arr = np.frombuffer(bytes(b), dtype=np.uint8)
        return ctypes.c_void_p(arr.ctypes.data), arr
    raise TypeError(type(b))


def device_count() -> int:
    n = ctypes.c_int(0)
    check(lib().mi_device_count(ctypes.byref(n)))
    return n.value


class Context:
    def __init__(self, device: int = 0):
        self.h = ctypes.c_void_p()
        check(lib().mi_ctx_create(device, ctypes.byref(self.h)))
        self.device = device

    def close(self):
        if self.h:
            lib().mi_ctx_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        check(lib().mi_ctx_synchronize(self.h))

    def stream(self) -> int:
        s = ctypes.c_void_p()
        check(lib().mi_ctx_stream(self.h, ctypes.byref(s)))
        return s.value or 0

    # ---- device timers (HIP events inside the library; always on) ----
    STAT_KEYS = ["accum_g1", "accum_g2", "msm_g1", "msm_g2", "sort", "ntt", "prove", "h2d", "poseidon", "tree_h2d",
                 "wit_a", "wit_sha", "wit_pos"]

    def reset_stats(self):
        check(lib().mi_ctx_reset_stats(self.h))

    def stats(self) -> dict:
        out = (ctypes.c_double * (3 * len(self.STAT_KEYS)))()
        check(lib().mi_ctx_get_stats(self.h, out))
        v = list(out)
        st = {k: {"ms": v[3 * i], "launches": int(v[3 * i + 1]), "units": int(v[3 * i + 2])}
              for i, k in enumerate(self.STAT_KEYS)}
        w = (ctypes.c_uint64 * 2)()
        check(lib().mi_ctx_get_work(self.h, w))
        st["accum_g1"]["madds"], st["accum_g2"]["madds"] = int(w[0]), int(w[1])
        return st

    def fallbacks(self) -> dict:
        """proofs re-run after an out-of-memory error with their key's split tables released, since the last
        reset_stats (mi_ctx_get_fallbacks)"""
        w = (ctypes.c_uint64 * 2)()
        check(lib().mi_ctx_get_fallbacks(self.h, w))
        return {"oom_retries": int(w[0]), "freed_bytes": int(w[1])}

    def shared_plans(self) -> int:
        """proofs since the last reset_stats whose L and A MSMs shared one plan (mi_ctx_get_shared_plans)"""
        w = ctypes.c_uint64(0)
        check(lib().mi_ctx_get_shared_plans(self.h, ctypes.byref(w)))
        return int(w.value)

    def derived_plans(self) -> int:
        """proofs since the last reset_stats whose A plan was filtered out of L's (mi_ctx_get_derived_plans)"""
        w = ctypes.c_uint64(0)
        check(lib().mi_ctx_get_derived_plans(self.h, ctypes.byref(w)))
        return int(w.value)

    def table_msms(self, g2: bool = False) -> int:
        """G1 (G2 with g2) MSMs that ran over a fixed-base window table since the last reset_stats
        (mi_ctx_get_table_msms)"""
        w = (ctypes.c_uint64 * 2)()
        check(lib().mi_ctx_get_table_msms(self.h, w))
        return int(w[1] if g2 else w[0])

    def inject_oom(self, count: int):
        """TEST ONLY (mi_ctx_inject_oom): the first attempt of each of the next ``count`` proofs fails with a real
        out-of-memory error after the NTT chain (-1: every proof, 0: off)"""
        check(lib().mi_ctx_inject_oom(self.h, int(count)))

    # ---- building blocks ----
    def msm_g1(self, bases96: bytes, scalars32: bytes) -> bytes:
        n = len(scalars32) // 32
        assert len(bases96) >= 96 * n
        out = ctypes.create_string_buffer(96)
        check(lib().mi_msm_g1(self.h, bytes(bases96), bytes(scalars32), n, out))
        return out.raw

    def msm_g2(self, bases192: bytes, scalars32: bytes) -> bytes:
        n = len(scalars32) // 32
        assert len(bases192) >= 192 * n
        out = ctypes.create_string_buffer(192)
        check(lib().mi_msm_g2(self.h, bytes(bases192), bytes(scalars32), n, out))
        return out.raw

    def ntt(self, data32: bytes, log_n: int, inverse=False, coset=False) -> bytes:
        assert len(data32) == 32 << log_n
        buf = ctypes.create_string_buffer(bytes(data32), len(data32))
        check(lib().mi_ntt_fr(self.h, buf, log_n, int(inverse), int(coset)))
        return buf.raw

    def ntt_dev(self, data_ptr: int, log_n: int, inverse=False, coset=False):
        torch_sync(self)
        check(lib().mi_ntt_fr_dev(self.h, ctypes.c_void_p(data_ptr), log_n, int(inverse), int(coset)))


class Points:
    """Device-resident MSM bases (uploaded once, like the resident SRS)."""

    def __init__(self, ctx: Context, data: bytes = None, g2=False, _handle=None, n=None):
        self.ctx, self.g2 = ctx, g2
        if _handle is not None:
            self.h = _handle
        else:
            self.h = ctypes.c_void_p()
            esz = 192 if g2 else 96
            n = len(data) // esz
            f = lib().mi_points_upload_g2 if g2 else lib().mi_points_upload_g1
            check(f(ctx.h, bytes(data), n, ctypes.byref(self.h)))
        self.n = lib().mi_points_count(self.h)

    def check_subgroup(self):
        """r P == O for every base (raises FilGpuError otherwise); marks the bases subgroup-known, which
        lets large G1 MSMs over them take the GLV split."""
        check(lib().mi_points_check_subgroup(self.ctx.h, self.h))

    def info(self):
        """{"count", "split_table", "subgroup"}"""
        out = (ctypes.c_uint64 * 3)()
        check(lib().mi_points_info(self.h, out))
        return {"count": out[0], "split_table": bool(out[1]), "subgroup": bool(out[2])}

    def precompute(self, window_bits: int = 0, n_points: int = None):
        """Fixed-base window table of the first n_points bases (mi_points_precompute): later G1 MSMs over at most
        n_points scalars run every window into one bucket set.  window_bits 0 = the library's choice."""
        check(lib().mi_points_precompute(self.ctx.h, self.h, int(window_bits), int(self.n if n_points is None else n_points)))

    def table_info(self):
        """{"window_bits", "windows", "points"} of the window table (zeros without one)"""
        out = (ctypes.c_uint64 * 3)()
        check(lib().mi_points_table_info(self.h, out))
        return {"window_bits": int(out[0]), "windows": int(out[1]), "points": int(out[2])}

    def msm_dev(self, scalars_ptr: int, n: int) -> bytes:
        out = ctypes.create_string_buffer(192 if self.g2 else 96)
        f = lib().mi_msm_g2_dev if self.g2 else lib().mi_msm_g1_dev
        torch_sync(self.ctx)
        check(f(self.ctx.h, self.h, ctypes.c_void_p(scalars_ptr), n, out))
        return out.raw

    def __del__(self):
        try:
            lib().mi_points_free(self.h)
        except Exception:
            pass


class _R1CS(ctypes.Structure):
    _fields_ = [
        ("num_constraints", ctypes.c_uint64),
        ("num_inputs", ctypes.c_uint64),
        ("num_aux", ctypes.c_uint64),
        ("row_ptr", ctypes.c_void_p * 3),
        ("col", ctypes.c_void_p * 3),
        ("coeff", ctypes.c_void_p * 3),
    ]


class Circuit:
    """R1CS uploaded once per shape.  mats: 3 x (row_ptr u64[n+1], col u32[nnz], coeff u8[nnz*32])."""

    def __init__(self, ctx: Context, num_constraints: int, num_inputs: int, num_aux: int, mats):
        self.ctx = ctx
        keep = [(np.ascontiguousarray(rp, dtype=np.uint64), np.ascontiguousarray(c, dtype=np.uint32),
                 np.ascontiguousarray(k, dtype=np.uint8)) for rp, c, k in mats]
        s = _R1CS()
        s.num_constraints, s.num_inputs, s.num_aux = num_constraints, num_inputs, num_aux
        for m, (rp, c, k) in enumerate(keep):
            s.row_ptr[m] = rp.ctypes.data
            s.col[m] = c.ctypes.data if len(c) else None
            s.coeff[m] = k.ctypes.data if len(k) else None
        self.h = ctypes.c_void_p()
        check(lib().mi_circuit_load(ctx.h, ctypes.byref(s), ctypes.byref(self.h)))
        self._info()

    @classmethod
    def from_handle(cls, ctx: Context, h):
        """wrap a circuit the library uploaded itself (mi_stacked_load)"""
        self = cls.__new__(cls)
        self.ctx, self.h = ctx, h
        self._info()
        return self

    def _info(self):
        info = (ctypes.c_uint64 * 9)()
        check(lib().mi_circuit_info(self.h, info))
        (self.num_constraints, self.num_inputs, self.num_aux, self.d, self.n_a, self.n_b,
         *self.nnz) = list(info)

    @property
    def num_vars(self):
        return self.num_inputs + self.num_aux

    def __del__(self):
        try:
            lib().mi_circuit_free(self.h)
        except Exception:
            pass


class _SrsHost(ctypes.Structure):
    _fields_ = [("vk", ctypes.c_void_p), ("ic", ctypes.c_void_p), ("n_ic", ctypes.c_uint64),
                ("h", ctypes.c_void_p), ("n_h", ctypes.c_uint64), ("l", ctypes.c_void_p), ("n_l", ctypes.c_uint64),
                ("a", ctypes.c_void_p), ("n_a", ctypes.c_uint64), ("b_g1", ctypes.c_void_p),
                ("n_b_g1", ctypes.c_uint64), ("b_g2", ctypes.c_void_p), ("n_b_g2", ctypes.c_uint64)]


class SrsStream:
    """A proving key arriving in chunks (ProvingKey.stream_begin)."""

    def __init__(self, ctx, handle):
        self.ctx, self.h = ctx, handle

    def part(self, which: int, first: int, data, n: int, on_device=False):
        if on_device:
            torch_sync(self.ctx)
            ptr, keep = ctypes.c_void_p(int(data)), None
        else:
            buf = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray)
                                       else data)
            ptr, keep = ctypes.c_void_p(buf.ctypes.data), buf
        check(lib().mi_srs_stream_part(self.h, which, first, ptr, n, int(on_device)))
        del keep

    def end(self):
        h, self.h = self.h, None
        hd = ctypes.c_void_p()
        check(lib().mi_srs_stream_end(h, ctypes.byref(hd)))
        return ProvingKey(self.ctx, hd)

    def abort(self):
        if self.h is not None:
            lib().mi_srs_stream_abort(self.h)
            self.h = None


class ProvingKey:
    """Device-resident Groth16 proving key (bellman layout)."""

    def __init__(self, ctx: Context, handle):
        self.ctx, self.h = ctx, handle
        info = (ctypes.c_uint64 * 6)()
        check(lib().mi_srs_info(self.h, info))
        self.d, self.n_h, self.n_l, self.n_a, self.n_b, self.n_ic = list(info)

    @classmethod
    def load(cls, ctx: Context, circuit, vk, ic, h, l, a, b_g1, b_g2, checked=False):
        keep = []

        def p(b):
            ptr, k = _ptr(b) if len(b) else (None, None)
            keep.append(k)
            return ptr

        s = _SrsHost()
        s.vk, s.ic, s.n_ic = p(vk), p(ic), len(ic) // 96
        s.h, s.n_h = p(h), len(h) // 96
        s.l, s.n_l = p(l), len(l) // 96
        s.a, s.n_a = p(a), len(a) // 96
        s.b_g1, s.n_b_g1 = p(b_g1), len(b_g1) // 96
        s.b_g2, s.n_b_g2 = p(b_g2), len(b_g2) // 192
        hd = ctypes.c_void_p()
        check(lib().mi_srs_load(ctx.h, circuit.h if circuit is not None else None, ctypes.byref(s), int(checked),
                                ctypes.byref(hd)))
        return cls(ctx, hd)

    @classmethod
    def load_params(cls, ctx: Context, circuit, path: str, checked=True):
        """Upload a bellman / filecoin ``v28-*.params`` file (mmapped, streamed to the device) --
        read_cached_params / get_groth_params (core/parameter_cache.hpp:125-129,185-200)."""
        hd = ctypes.c_void_p()
        check(lib().mi_params_load(ctx.h, circuit.h if circuit is not None else None, os.fsencode(path),
                                   int(checked), ctypes.byref(hd)))
        return cls(ctx, hd)

    def write_params(self, path: str):
        """bellman Parameters::write (write_cached_params, core/parameter_cache.hpp:146-152)."""
        check(lib().mi_params_write(self.ctx.h, self.h, os.fsencode(path)))

    def write_vk(self, path: str):
        """bellman VerifyingKey::write (write_cached_verifying_key, core/parameter_cache.hpp:136-144)."""
        check(lib().mi_vk_write(self.h, os.fsencode(path)))

    @classmethod
    def stream_begin(cls, ctx: Context, circuit, vk: bytes, ic: bytes, counts, checked=False):
        """Streaming key load (mi_srs_stream_*): counts = |h|, |l|, |a|, |b_g1|, |b_g2|; feed every query in
        order with .part(which, first, data, n, on_device) and finish with .end() -> ProvingKey."""
        hd = ctypes.c_void_p()
        arr = (ctypes.c_uint64 * 5)(*counts)
        check(lib().mi_srs_stream_begin(ctx.h, circuit.h if circuit is not None else None, bytes(vk), bytes(ic),
                                        len(ic) // 96, arr, int(checked), ctypes.byref(hd)))
        return SrsStream(ctx, hd)

    def export_query_dev(self, which: int, first: int, n: int, dev_ptr: int):
        """points [first, first + n) of one query (0 h natural order, 1 l, 2 a, 3 b_g1, 4 b_g2) in the wire
        format, written to device memory"""
        torch_sync(self.ctx)
        check(lib().mi_srs_export_query_dev(self.ctx.h, self.h, which, first, n, ctypes.c_void_p(dev_ptr)))

    def msm_info(self):
        """{"split_tables": 2^128 tables of h, l, a resident, "subgroup": every point subgroup-known}.
        A subgroup-known key without tables runs its split-size G1 MSMs through GLV."""
        out = (ctypes.c_uint64 * 2)()
        check(lib().mi_srs_msm_info(self.h, out))
        return {"split_tables": bool(out[0]), "subgroup": bool(out[1])}

    def table_state(self):
        """{"split_tables", "dropped": out-of-memory releases since the tables were last built, "subgroup"}"""
        out = (ctypes.c_uint64 * 3)()
        check(lib().mi_srs_table_state(self.h, out))
        return {"split_tables": bool(out[0]), "dropped": int(out[1]), "subgroup": bool(out[2])}

    def shared_la(self) -> bool:
        """True when the key holds its A query in the aux index space: whole proofs run L and A over one plan
        (mi_srs_shared_la)"""
        v = ctypes.c_int(0)
        check(lib().mi_srs_shared_la(self.h, ctypes.byref(v)))
        return bool(v.value)

    def window_tables(self):
        """{"window_bits", "windows", "queries"}: the fixed-base window tables of a small key (mi_srs_window_tables)"""
        out = (ctypes.c_uint64 * 3)()
        check(lib().mi_srs_window_tables(self.h, out))
        return {"window_bits": int(out[0]), "windows": int(out[1]), "queries": int(out[2])}

    def readmit(self) -> int:
        """rebuilds split tables an out-of-memory release took, once they fit again (mi_srs_readmit); returns the
        table bytes rebuilt"""
        got = ctypes.c_uint64()
        check(lib().mi_srs_readmit(self.ctx.h, self.h, ctypes.byref(got)))
        return int(got.value)

    def verifying_key(self):
        vk = ctypes.create_string_buffer(VK_BYTES)
        ic = ctypes.create_string_buffer(96 * self.n_ic)
        check(lib().mi_srs_export_vk(self.h, vk, ic))
        return vk.raw, ic.raw

    def query(self, which: int) -> bytes:
        n = {0: self.n_h, 1: self.n_l, 2: self.n_a, 3: self.n_b, 4: self.n_b}[which]
        esz = 192 if which == 4 else 96
        out = ctypes.create_string_buffer(max(1, esz * n))
        check(lib().mi_srs_export_query(self.ctx.h, self.h, which, out, n))
        return out.raw[: esz * n]

    def points(self, which: int) -> Points:
        hd = ctypes.c_void_p()
        check(lib().mi_points_from_srs(self.ctx.h, self.h, which, ctypes.byref(hd)))
        p = Points(self.ctx, g2=(which == 4), _handle=hd)
        p._srs = self  # keep the key alive while the borrowed points live
        return p

    def __del__(self):
        try:
            lib().mi_srs_free(self.h)
        except Exception:
            pass


def verify(vk: bytes, ic: bytes, inputs: bytes, proof: bytes) -> bool:
    """bellman verify_proof on the host (the C2 self-check, api/seal.hpp:310-313).  ``inputs`` are the
    public inputs without the implicit ONE, 32 B LE each (len(ic) / 96 - 1 of them)."""
    n_ic = len(ic) // 96
    assert len(vk) == VK_BYTES and len(inputs) == 32 * (n_ic - 1) and len(proof) == PROOF_BYTES
    ok = ctypes.c_int(0)
    check(lib().mi_groth16_verify(vk, ic, n_ic, inputs or None, proof, ctypes.byref(ok)))
    return bool(ok.value)


def verify_batch(vk: bytes, ic: bytes, inputs, proofs, seed: bytes = None) -> bool:
    """bellman verify_proofs_batch (verify_batch_seal, api/seal.hpp:339-485): one multi-pairing with
    random 128-bit weights from getrandom() (bellman: OsRng).  ``seed`` (32 B, tests only) makes the
    weights a reproducible ChaCha20 stream instead (mi_groth16_verify_batch_seeded)."""
    n_ic = len(ic) // 96
    assert len(inputs) == len(proofs) and all(len(x) == 32 * (n_ic - 1) for x in inputs)
    assert seed is None or len(seed) == 32
    ok = ctypes.c_int(0)
    ins, prs = b"".join(inputs) or None, b"".join(proofs) or None
    if seed is None:
        check(lib().mi_groth16_verify_batch(vk, ic, n_ic, len(proofs), ins, prs, ctypes.byref(ok)))
    else:
        check(lib().mi_groth16_verify_batch_seeded(vk, ic, n_ic, len(proofs), ins, prs, bytes(seed),
                                                   ctypes.byref(ok)))
    return bool(ok.value)


def pairing(g1_96: bytes, g2_192: bytes) -> bytes:
    """Reduced optimal-ate pairing e(P, Q): 12 x 48 B big-endian Fq coefficients (w^0..w^5 basis)."""
    out = ctypes.create_string_buffer(576)
    check(lib().mi_pairing(bytes(g1_96), bytes(g2_192), out))
    return out.raw


def params_inspect(path: str) -> dict:
    """Vector lengths of a params file (no device needed): ic, h, l, a, b_g1, b_g2."""
    out = (ctypes.c_uint64 * 6)()
    check(lib().mi_params_inspect(os.fsencode(path), out))
    return dict(zip(("ic", "h", "l", "a", "b_g1", "b_g2"), list(out)))


# ---- parameter cache (core/parameter_cache.hpp:50-219; mi_param_cache_* / mi_get_groth_params) ----
PARAMS_VERSION = 28
PARAMS, META, VK = 0, 1, 2  # parameter_cache_{params,metadata,verifying_key}_path


def _cstr(f, *args) -> str:
    buf = ctypes.create_string_buffer(4096)
    check(f(*args, buf, len(buf)))
    return buf.value.decode()


def param_cache_id(cache_prefix: str, identifier: str) -> str:
    """cacheable_parameters::cache_identifier: "<cache_prefix>-<hex sha256(identifier)>" """
    return _cstr(lib().mi_param_cache_id, cache_prefix.encode(), identifier.encode())


def param_cache_path(cache_id: str, kind: int = PARAMS) -> str:
    """$FIL_PROOFS_PARAMETER_CACHE/v28-<id>.params / .meta / .vk"""
    return _cstr(lib().mi_param_cache_path, cache_id.encode(), int(kind))


def param_cache_metadata(cache_id: str, sector_size: int) -> int:
    """get_param_metadata: the cached sector size, written on first use"""
    out = ctypes.c_uint64()
    check(lib().mi_param_cache_metadata(cache_id.encode(), int(sector_size), ctypes.byref(out)))
    return int(out.value)


def get_groth_params(ctx: Context, circuit: Circuit, cache_id: str, toxic=None, checked=False):
    """get_groth_params: the cached key when <id>.params exists and parses, else a generated one (from ``toxic``,
    or OS randomness when None), written to the cache together with <id>.vk.  Returns (ProvingKey, generated)."""
    hd, gen = ctypes.c_void_p(), ctypes.c_int()
    tb = b"".join(fr_bytes(t) for t in toxic) if toxic is not None else None
    check(lib().mi_get_groth_params(ctx.h, circuit.h, cache_id.encode(), tb, int(checked), ctypes.byref(hd),
                                    ctypes.byref(gen)))
    return ProvingKey(ctx, hd), bool(gen.value)


def generate_random_parameters(ctx: Context, circuit: Circuit, toxic) -> ProvingKey:
    """GPU groth16::generate_random_parameters with known toxic waste (tau, alpha, beta, gamma, delta)."""
    tb = b"".join(fr_bytes(t) for t in toxic)
    hd = ctypes.c_void_p()
    check(lib().mi_srs_generate(ctx.h, circuit.h, tb, ctypes.byref(hd)))
    return ProvingKey(ctx, hd)


def prove(ctx: Context, pk: ProvingKey, circuit: Circuit, z, r: int = None, s: int = None, priority=False,
          want_raw=False):
    """One Groth16 proof. z: bytes (num_vars x 32 LE) or a device pointer (int) to the same layout.
    r = s = None: the production entry, blinding drawn inside the library from getrandom() (crypto3 prove /
    bellman create_random_proof); explicit r, s are the parity/test entry."""
    proof = ctypes.create_string_buffer(PROOF_BYTES)
    if r is None and s is None:
        if want_raw:
            raise ValueError("want_raw needs injected r, s")
        if isinstance(z, int):
            torch_sync(ctx)
            check(lib().mi_groth16_prove_dev_random(ctx.h, pk.h, circuit.h, ctypes.c_void_p(z), int(priority), proof))
        else:
            assert len(z) == 32 * circuit.num_vars, "witness length must be (num_inputs + num_aux) * 32"
            check(lib().mi_groth16_prove_random(ctx.h, pk.h, circuit.h, bytes(z), int(priority), proof))
        return proof.raw
    if r is None or s is None:
        raise ValueError("give both r and s, or neither")
    raw = ctypes.create_string_buffer(384) if want_raw else None
    if isinstance(z, int):
        torch_sync(ctx)
        check(lib().mi_groth16_prove_dev(ctx.h, pk.h, circuit.h, ctypes.c_void_p(z), fr_bytes(r), fr_bytes(s),
                                         int(priority), proof, raw))
    else:
        assert len(z) == 32 * circuit.num_vars, "witness length must be (num_inputs + num_aux) * 32"
        check(lib().mi_groth16_prove(ctx.h, pk.h, circuit.h, bytes(z), fr_bytes(r), fr_bytes(s), int(priority),
                                     proof, raw))
    return (proof.raw, raw.raw) if want_raw else proof.raw


class _PinnedAlloc:
    """Owner of one mi_host_alloc block; freed when the last view of it is gone."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        check(lib().mi_host_alloc(nbytes, ctypes.byref(p)))
        self.ptr = p.value

    def __del__(self):
        try:
            lib().mi_host_free(ctypes.c_void_p(self.ptr))
        except Exception:
            pass


class HostBuffer:
    """Page-locked host memory from mi_host_alloc: a witness written here goes to the GPU at full DMA
    rate (and prove_batch overlaps the next partition's copy with the current proof).  ``array`` owns the
    allocation through its base (a ctypes array holding the _PinnedAlloc), so a view that outlives the
    HostBuffer object keeps the pages alive instead of dangling."""

    def __init__(self, nbytes: int):
        owner = _PinnedAlloc(nbytes)
        self.ptr, self.nbytes = owner.ptr, nbytes
        cbuf = (ctypes.c_uint8 * nbytes).from_address(self.ptr)
        cbuf._owner = owner  # the numpy view -> cbuf -> owner chain keeps the allocation alive
        self.array = np.frombuffer(cbuf, dtype=np.uint8)


def _host_ptr(z, nbytes):
    """(address, keepalive) of a host witness without copying it: HostBuffer, numpy array or bytes.  A device
    pointer (int) is refused: the batch entry uploads host witnesses (use prove / circuit_proofs for those)."""
    if isinstance(z, int):
        raise TypeError("prove_batch takes host witnesses; a device pointer (int) goes through prove()")
    if isinstance(z, HostBuffer):
        assert z.nbytes >= nbytes
        return z.ptr, z
    if isinstance(z, np.ndarray):
        assert z.flags.c_contiguous and z.nbytes >= nbytes
        return z.ctypes.data, z
    b = bytes(z)
    assert len(b) >= nbytes
    arr = np.frombuffer(b, dtype=np.uint8)
    return arr.ctypes.data, arr


def prove_batch(ctx: Context, pk: ProvingKey, circuit: Circuit, zs, rs=None, priority=False):
    """count independent partition proofs -> list of 192-byte proofs.  Witnesses stay in host memory
    (HostBuffer, numpy arrays or bytes; never copied here): the library uploads partition k + 1 while
    it proves partition k.  rs = None: blinding drawn inside the library (mi_groth16_prove_batch_random)."""
    count = len(zs)
    nbytes = 32 * circuit.num_vars
    keep = [_host_ptr(z, nbytes) for z in zs]
    arr = (ctypes.c_void_p * count)(*[p for p, _ in keep])
    out = ctypes.create_string_buffer(PROOF_BYTES * count)
    if rs is None:
        check(lib().mi_groth16_prove_batch_random(ctx.h, pk.h, circuit.h, count, arr, int(priority), out))
        return [out.raw[i * PROOF_BYTES:(i + 1) * PROOF_BYTES] for i in range(count)]
    if len(rs) != count:
        raise ValueError("one (r, s) pair per partition is required")
    rsb = b"".join(fr_bytes(r) + fr_bytes(s) for r, s in rs)
    check(lib().mi_groth16_prove_batch(ctx.h, pk.h, circuit.h, count, arr, rsb, int(priority), out))
    return [out.raw[i * PROOF_BYTES:(i + 1) * PROOF_BYTES] for i in range(count)]


def h_coeffs_dev(ctx: Context, circuit: Circuit, z_dev_ptr: int, h_out_ptr: int):
    """mi_groth16_h_coeffs_dev: the witness map + NTT chain alone; writes d x 32 B canonical H coefficients (the
    key's bit-reversed h order) to device memory (a latency group's lead broadcasts them)"""
    torch_sync(ctx)
    check(lib().mi_groth16_h_coeffs_dev(ctx.h, circuit.h, ctypes.c_void_p(z_dev_ptr), ctypes.c_void_p(h_out_ptr)))


def prove_share_ranges(ctx: Context, pk: ProvingKey, circuit: Circuit, z, ranges, priority=False, h_dev=None) -> bytes:
    """A latency-mode share over explicit query ranges: ranges = [(first, count)] for H (d - 1 points, h order),
    L, A and B (B_G1 and B_G2); H is computed (witness map + NTT chain) only when its count is non-zero and no
    ``h_dev`` (device pointer to h_coeffs_dev's output) is given.  z as for ``prove`` (a device pointer when h_dev
    is given).  Shares whose ranges partition every query go to ``assemble`` (a rank may contribute several)."""
    flat = [int(v) for fc in ranges for v in fc]
    if len(flat) != 8:
        raise ValueError("four (first, count) ranges: H, L, A, B")
    arr = (ctypes.c_uint64 * 8)(*flat)
    out = ctypes.create_string_buffer(SHARE_BYTES)
    if h_dev is not None:
        if not isinstance(z, int):
            raise ValueError("h_dev needs a device witness pointer")
        torch_sync(ctx)
        check(lib().mi_groth16_prove_share_ranges_h_dev(ctx.h, pk.h, circuit.h, ctypes.c_void_p(z),
                                                        ctypes.c_void_p(h_dev), arr, int(priority), out))
        return out.raw
    if isinstance(z, int):
        torch_sync(ctx)
        check(lib().mi_groth16_prove_share_ranges_dev(ctx.h, pk.h, circuit.h, ctypes.c_void_p(z), arr, int(priority),
                                                      out))
    else:
        assert len(z) == 32 * circuit.num_vars, "witness length must be (num_inputs + num_aux) * 32"
        check(lib().mi_groth16_prove_share_ranges(ctx.h, pk.h, circuit.h, bytes(z), arr, int(priority), out))
    return out.raw


def prove_share(ctx: Context, pk: ProvingKey, circuit: Circuit, z, rank: int, world: int, priority=False) -> bytes:
    """Single-proof latency mode: this rank's share of the five MSMs of one proof
    (SHARE_BYTES). z as for ``prove``. The shares of ranks 0..world-1 go to ``assemble``."""
    out = ctypes.create_string_buffer(SHARE_BYTES)
    if isinstance(z, int):
        torch_sync(ctx)
        check(lib().mi_groth16_prove_share_dev(ctx.h, pk.h, circuit.h, ctypes.c_void_p(z), rank, world,
                                               int(priority), out))
    else:
        assert len(z) == 32 * circuit.num_vars, "witness length must be (num_inputs + num_aux) * 32"
        check(lib().mi_groth16_prove_share(ctx.h, pk.h, circuit.h, bytes(z), rank, world, int(priority), out))
    return out.raw


def assemble(vk: bytes, shares, r: int, s: int, want_raw=False):
    """Add the ranks' shares and blind: the proof ``prove`` returns for the same (z, r, s). Host only."""
    shares = [bytes(x) for x in shares]
    if not shares or any(len(x) != SHARE_BYTES for x in shares):
        raise ValueError(f"shares are {SHARE_BYTES} bytes each, at least one")
    assert len(vk) == VK_BYTES
    proof = ctypes.create_string_buffer(PROOF_BYTES)
    raw = ctypes.create_string_buffer(384) if want_raw else None
    check(lib().mi_groth16_assemble(bytes(vk), b"".join(shares), len(shares), fr_bytes(r), fr_bytes(s), proof, raw))
    return (proof.raw, raw.raw) if want_raw else proof.raw


def trapdoor_dlogs(ctx: Context, pk: ProvingKey, circuit: Circuit, z_dev_ptr: int, r: int, s: int):
    out = ctypes.create_string_buffer(96)
    torch_sync(ctx)
    check(lib().mi_groth16_trapdoor_dlogs(ctx.h, pk.h, circuit.h, ctypes.c_void_p(z_dev_ptr), fr_bytes(r),
                                          fr_bytes(s), out))
    return [int.from_bytes(out.raw[32 * i:32 * i + 32], "little") for i in range(3)]


def msm_window_bits(n: int) -> int:
    return lib().mi_msm_window_bits(n)
