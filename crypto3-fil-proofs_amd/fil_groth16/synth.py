"""Synthetic BASELINE workloads (configs 3/4): a satisfiable R1CS of 2^log_rows - n_in rows and its
witness, generated deterministically by the library's multithreaded host generator
(csrc/synth.hip).  Circuit synthesis is outside the prover boundary in the reference
(StackedCircuit::synthesize, porep/stacked/circuit/proof.hpp:98-165); this stands in for it."""
import ctypes

import numpy as np

from ._lib import check, lib
from .core import Circuit, _R1CS


class SynthCircuit:
    def __init__(self, log_rows: int, n_in: int = 4, seed: int = 1, uniform: bool = False):
        """uniform: no boolean rows, so every witness value is uniform (MI_SYNTH_UNIFORM_WITNESS); the default
        mixes boolean, random and product rows like a Filecoin witness"""
        self.h = ctypes.c_void_p()
        check(lib().mi_synth_generate_ex(log_rows, n_in, seed, 1 if uniform else 0, ctypes.byref(self.h)))
        self.uniform = uniform
        self.s = _R1CS()
        check(lib().mi_synth_r1cs(self.h, ctypes.byref(self.s)))
        zp, nv = ctypes.c_void_p(), ctypes.c_uint64()
        check(lib().mi_synth_witness(self.h, ctypes.byref(zp), ctypes.byref(nv)))
        self._z_ptr, self.num_vars = zp.value, nv.value
        self.log_rows = log_rows
        self.n = self.s.num_constraints
        self.n_in = self.s.num_inputs
        self.n_aux = self.s.num_aux

    def z_array(self) -> np.ndarray:
        """zero-copy uint8 view of the witness (num_vars x 32 bytes, canonical LE Fr)"""
        buf = (ctypes.c_uint8 * (32 * self.num_vars)).from_address(self._z_ptr)
        return np.frombuffer(buf, dtype=np.uint8)

    def z_bytes(self) -> bytes:
        return self.z_array().tobytes()

    def csr(self):
        """numpy views of the CSR matrices: 3 x (row_ptr u64, col u32, coeff u8[nnz*32])"""
        mats = []
        for m in range(3):
            rp = np.ctypeslib.as_array((ctypes.c_uint64 * (self.n + 1)).from_address(self.s.row_ptr[m]))
            nnz = int(rp[-1])
            col = np.ctypeslib.as_array((ctypes.c_uint32 * max(nnz, 1)).from_address(self.s.col[m]))[:nnz]
            co = np.ctypeslib.as_array((ctypes.c_uint8 * max(32 * nnz, 1)).from_address(self.s.coeff[m]))[: 32 * nnz]
            mats.append((rp, col, co))
        return mats

    def load(self, ctx) -> Circuit:
        return Circuit(ctx, self.n, self.n_in, self.n_aux, self.csr())

    def __del__(self):
        try:
            lib().mi_synth_free(self.h)
        except Exception:
            pass
