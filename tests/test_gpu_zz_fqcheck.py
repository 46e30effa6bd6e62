"""the device Fq magnitude invariant, checked on the device once.

Meaningful only with the MI_FQ_CHECK debug build of the library (`make -C crypto3-fil-proofs_amd fqcheck`, loaded with
FILGPU_LIB=crypto3-fil-proofs_amd/build_fqcheck/libfilgpu.so) and run AFTER the MSM / window-table / prove parity tests
in the same process, e.g.

    FILGPU_LIB=crypto3-fil-proofs_amd/build_fqcheck/libfilgpu.so python -m pytest -m gpu \\
        tests/test_gpu_kernels.py tests/test_gpu_groth16.py tests/test_gpu_zz_fqcheck.py

The debug build counts, in every kernel of every translation unit, normalised Fq values whose top limb exceeds 2^24
(|V| beyond ~9.8 p) and zero tests with |round(V / p)| > 3 (csrc/field.h).  The first bound is the hard one
(fq_quot, and with it fq_is_zero, is exact only below it); the second is the MSM group law's property, which the
key-table doubling chains of prover.hip exceed (|k| = 4, 1,694 times in the round-6 run, handled by fq_is_zero's
reduction loop), so it is reported, not asserted.  The per-unit counts go to stderr.  With the release library (no
counters) the test is skipped."""
import ctypes

import pytest

from fil_groth16._lib import lib

pytestmark = pytest.mark.gpu


def test_fq_magnitude_invariant_held(ctx):
    out = (ctypes.c_uint64 * 2)()
    if lib().mi_fq_check_read(out, 0) != 0:
        pytest.skip("release library: built without MI_FQ_CHECK")
    assert out[0] == 0, f"normalised values with |top limb| > 2^24: {out[0]}"
    print(f"[fq-check] top-limb violations {out[0]}, zero-test violations {out[1]}", flush=True)
