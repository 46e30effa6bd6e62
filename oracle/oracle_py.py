"""ctypes binding for the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker.  The product package never imports this module.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB selects another build of the same sources, e.g. the ASan/UBSan one (make -C oracle asan)
LIB_PATH = os.environ.get("ORACLE_LIB", os.path.join(_HERE, "build", "liboracle.so"))

R_MOD = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
P_MOD = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB

_lib = None


def build():
    import subprocess

    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.c_char_p
        L.or_groth16_keygen.restype = ctypes.c_void_p
        L.or_groth16_keygen.argtypes = [ctypes.c_void_p, u8p]
        L.or_params_free.argtypes = [ctypes.c_void_p]
        L.or_params_from_queries.restype = ctypes.c_void_p
        L.or_params_from_queries.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint64, u8p, u8p, ctypes.c_uint64, u8p,
                                             u8p, ctypes.c_uint64, u8p, u8p]
        L.or_params_sizes.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.or_params_export.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 7
        L.or_groth16_prove.argtypes = [ctypes.c_void_p, ctypes.c_void_p, u8p, u8p, u8p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p]
        L.or_groth16_trapdoor_check.argtypes = [ctypes.c_void_p, ctypes.c_void_p, u8p, u8p, u8p, u8p]
        L.or_groth16_verify.argtypes = [u8p, u8p, ctypes.c_uint64, u8p, u8p]
        L.or_r1cs_satisfied.argtypes = [ctypes.c_void_p, u8p]
        L.or_ntt.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_int]
        for f in ("or_msm_g1", "or_msm_g2", "or_msm_g1_naive"):
            getattr(L, f).argtypes = [u8p, u8p, ctypes.c_size_t, ctypes.c_void_p]
        L.or_g1_fixed_base.argtypes = [u8p, ctypes.c_size_t, ctypes.c_void_p]
        L.or_g2_fixed_base.argtypes = [u8p, ctypes.c_size_t, ctypes.c_void_p]
        L.or_set_threads.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


# ------------------------------------------------------------------ encodings
def fr_bytes(x):
    return int(x % R_MOD).to_bytes(32, "little")


def fr_vec_bytes(xs):
    return b"".join(fr_bytes(x) for x in xs)


def fr_from_bytes(b):
    return int.from_bytes(b, "little")


def _buf(n):
    return ctypes.create_string_buffer(n)


def g1_generator():
    b = _buf(96)
    lib().or_g1_generator(b)
    return b.raw


def g2_generator():
    b = _buf(192)
    lib().or_g2_generator(b)
    return b.raw


def g1_mul(p, s):
    b = _buf(96)
    assert lib().or_g1_mul(p, fr_bytes(s) if isinstance(s, int) else s, b) == 0
    return b.raw


def g2_mul(p, s):
    b = _buf(192)
    assert lib().or_g2_mul(p, fr_bytes(s) if isinstance(s, int) else s, b) == 0
    return b.raw


def g1_add(a, c):
    b = _buf(96)
    assert lib().or_g1_add(a, c, b) == 0
    return b.raw


def g2_add(a, c):
    b = _buf(192)
    assert lib().or_g2_add(a, c, b) == 0
    return b.raw


def g1_compress(p):
    b = _buf(48)
    assert lib().or_g1_compress(p, b) == 0
    return b.raw


def g2_compress(p):
    b = _buf(96)
    assert lib().or_g2_compress(p, b) == 0
    return b.raw


def g1_fixed_base(ks):
    kb = fr_vec_bytes(ks) if not isinstance(ks, (bytes, bytearray)) else bytes(ks)
    n = len(kb) // 32
    out = _buf(96 * n)
    lib().or_g1_fixed_base(kb, n, out)
    return out.raw


def g2_fixed_base(ks):
    kb = fr_vec_bytes(ks) if not isinstance(ks, (bytes, bytearray)) else bytes(ks)
    n = len(kb) // 32
    out = _buf(192 * n)
    lib().or_g2_fixed_base(kb, n, out)
    return out.raw


def ntt(data: bytes, log_n: int, kind: int) -> bytes:
    """kind: 0 fft, 1 ifft, 2 coset_fft, 3 icoset_fft (bellman EvaluationDomain semantics)."""
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    lib().or_ntt(buf, log_n, kind)
    return buf.raw


def msm_g1(bases: bytes, scalars: bytes) -> bytes:
    n = len(scalars) // 32
    out = _buf(96)
    assert lib().or_msm_g1(bases, scalars, n, out) == 0
    return out.raw


def msm_g1_naive(bases: bytes, scalars: bytes) -> bytes:
    n = len(scalars) // 32
    out = _buf(96)
    assert lib().or_msm_g1_naive(bases, scalars, n, out) == 0
    return out.raw


def msm_g2(bases: bytes, scalars: bytes) -> bytes:
    n = len(scalars) // 32
    out = _buf(192)
    assert lib().or_msm_g2(bases, scalars, n, out) == 0
    return out.raw


def set_threads(n):
    lib().or_set_threads(n)


def poseidon_hash(arity: int, preimages: bytes) -> bytes:
    """C restatement of oracle/poseidon_ref.py (literal rounds, OpenMP): digests of consecutive groups of
    `arity` canonical 32-byte LE inputs."""
    import poseidon_ref as P

    h = P.poseidon(arity)
    rc = b"".join(P.fr_to_bytes(x) for x in h.rc)
    mds = b"".join(P.fr_to_bytes(x) for row in h.m for x in row)
    n = len(preimages) // (32 * arity)
    out = _buf(32 * max(n, 1))
    L = lib()
    L.or_poseidon_hash.argtypes = [ctypes.c_uint, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint, ctypes.c_uint,
                                   ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p]
    rc_ = L.or_poseidon_hash(arity, rc, mds, h.r_f, h.r_p, bytes(preimages), n, out)
    if rc_ != 0:
        raise ValueError("non-canonical Poseidon input")
    return out.raw[:32 * n]


def sha256(msg: bytes) -> bytes:
    """The oracle's FIPS 180-4 SHA-256 restatement (pinned against hashlib in the CPU tests)."""
    L = lib()
    L.or_sha256.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p]
    out = _buf(32)
    L.or_sha256(bytes(msg), len(msg), out)
    return out.raw


def sdr_labels(replica_id: bytes, layers, nodes, parents: bytes, n_parents: int) -> bytes:
    """SDR labelling witness (oracle.cpp or_sdr_labels): one 32-byte label per (layer, node), parents given
    as n_parents labels per entry and repeated cyclically to 37 (vanilla/proof.hpp:233-237)."""
    import numpy as _np

    lay = _np.ascontiguousarray(layers, dtype=_np.uint32)
    nod = _np.ascontiguousarray(nodes, dtype=_np.uint64)
    n = len(lay)
    assert len(nod) == n and len(replica_id) == 32 and len(parents) == 32 * n_parents * n
    L = lib()
    L.or_sdr_labels.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p,
                                ctypes.c_uint, ctypes.c_void_p]
    out = _buf(32 * max(n, 1))
    if L.or_sdr_labels(bytes(replica_id), n, lay.ctypes.data, nod.ctypes.data, bytes(parents), n_parents, out) != 0:
        raise ValueError("n_parents must be <= 37")
    return out.raw[:32 * n]


_SPARSE = {}


def poseidon_hash_sparse(arity: int, preimages: bytes) -> bytes:
    """The same digests through the C oracle's sparse (optimised) form, constants from
    poseidon_ref.sparse_form: the CPU baseline of the tree builders."""
    import poseidon_ref as P

    if arity not in _SPARSE:
        first, part, last, rows, dense = P.sparse_form(arity)
        h = P.poseidon(arity)
        enc = lambda xs: b"".join(P.fr_to_bytes(x) for x in xs)
        _SPARSE[arity] = (h.r_f, h.r_p, enc([x for r in first for x in r]), enc(part), enc([x for r in last for x in r]),
                          enc([x for row in h.m for x in row]), enc([x for row, w in rows for x in row + w]),
                          enc([x for row in dense for x in row]))
    rf, rp, first, part, last, mds, rows, dense = _SPARSE[arity]
    n = len(preimages) // (32 * arity)
    out = _buf(32 * max(n, 1))
    L = lib()
    L.or_poseidon_hash_sparse.argtypes = [ctypes.c_uint, ctypes.c_uint, ctypes.c_uint] + [ctypes.c_char_p] * 7 + [
        ctypes.c_uint64, ctypes.c_void_p]
    if L.or_poseidon_hash_sparse(arity, rf, rp, first, part, last, mds, rows, dense, bytes(preimages), n, out) != 0:
        raise ValueError("non-canonical Poseidon input")
    return out.raw[:32 * n]


# ------------------------------------------------------------------ R1CS / Groth16
class R1CS(ctypes.Structure):
    _fields_ = [
        ("num_constraints", ctypes.c_uint64),
        ("num_inputs", ctypes.c_uint64),
        ("num_aux", ctypes.c_uint64),
        ("row_ptr", ctypes.c_void_p * 3),
        ("col", ctypes.c_void_p * 3),
        ("coeff", ctypes.c_void_p * 3),
    ]


class OracleCircuit:
    """Holds numpy-backed CSR arrays alive for the oracle's or_r1cs view.

    mats: list of 3 (row_ptr uint64[n+1], col uint32[nnz], coeff uint8[nnz*32]).
    """

    def __init__(self, num_constraints, num_inputs, num_aux, mats):
        self.mats = [(np.ascontiguousarray(rp, dtype=np.uint64), np.ascontiguousarray(c, dtype=np.uint32),
                      np.ascontiguousarray(k, dtype=np.uint8)) for rp, c, k in mats]
        self.s = R1CS()
        self.s.num_constraints = num_constraints
        self.s.num_inputs = num_inputs
        self.s.num_aux = num_aux
        for m, (rp, c, k) in enumerate(self.mats):
            self.s.row_ptr[m] = rp.ctypes.data
            self.s.col[m] = c.ctypes.data
            self.s.coeff[m] = k.ctypes.data

    @property
    def ptr(self):
        return ctypes.byref(self.s)

    def satisfied(self, z: bytes) -> bool:
        return bool(lib().or_r1cs_satisfied(self.ptr, z))


class OracleParams:
    def __init__(self, circ: OracleCircuit, toxic=None, queries=None):
        """toxic: keygen from known toxic waste; queries: dict(h,l,a,b_g1,b_g2,vk,ic) wire bytes."""
        self.circ = circ
        if queries is not None:
            q = queries
            self.p = lib().or_params_from_queries(circ.ptr, q["h"], len(q["h"]) // 96, q["l"], q["a"],
                                                  len(q["a"]) // 96, q["b_g1"], q["b_g2"], len(q["b_g1"]) // 96,
                                                  q["vk"], q["ic"])
            if not self.p:
                raise ValueError("oracle could not load the given params")
        else:
            tb = b"".join(fr_bytes(t) for t in toxic)
            self.p = lib().or_groth16_keygen(circ.ptr, tb)
        sizes = (ctypes.c_uint64 * 6)()
        lib().or_params_sizes(self.p, sizes)
        self.d, self.nh, self.nl, self.na, self.nb1, self.nb2 = list(sizes)

    def export(self):
        h, l, a = _buf(96 * self.nh), _buf(96 * max(self.nl, 1)), _buf(96 * max(self.na, 1))
        b1, b2 = _buf(96 * max(self.nb1, 1)), _buf(192 * max(self.nb2, 1))
        vk = _buf(864)
        ic = _buf(96 * self.circ.s.num_inputs)
        lib().or_params_export(self.p, h, l, a, b1, b2, vk, ic)
        return dict(h=h.raw, l=l.raw[: 96 * self.nl], a=a.raw[: 96 * self.na], b_g1=b1.raw[: 96 * self.nb1],
                    b_g2=b2.raw[: 192 * self.nb2], vk=vk.raw, ic=ic.raw)

    def prove(self, z: bytes, r: int, s: int, want_h=False):
        proof, raw = _buf(192), _buf(384)
        hb = _buf(32 * (self.d - 1)) if want_h else None
        rc = lib().or_groth16_prove(self.p, self.circ.ptr, z, fr_bytes(r), fr_bytes(s), proof, raw, hb)
        assert rc == 0, rc
        return (proof.raw, raw.raw, hb.raw if want_h else None)

    def trapdoor_check(self, z: bytes, r: int, s: int, raw: bytes) -> bool:
        return bool(lib().or_groth16_trapdoor_check(self.p, self.circ.ptr, z, fr_bytes(r), fr_bytes(s), raw))

    def __del__(self):
        try:
            lib().or_params_free(self.p)
        except Exception:
            pass


def groth16_verify(vk: bytes, ic: bytes, inputs: bytes, raw: bytes) -> bool:
    n = len(inputs) // 32
    rc = lib().or_groth16_verify(vk, ic, n, inputs, raw)
    assert rc >= 0, rc
    return rc == 1
