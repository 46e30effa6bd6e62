"""Test / benchmark A/B switches of libfilgpu (mi_tune_set / mi_tune_clear / mi_tune_get; csrc/tune.h).

TEST ONLY.  Every switch defaults to the measured production choice and the library reads no environment
variable for them, so a production prove never changes window sizes, lanes or kernels behind its caller's back.
Tests and bench.py's A/B legs select a variant explicitly:

    with tuned(msm_split=2, msm_glv=1):
        ...

Values are process-wide (one table in the library); `tuned` restores what was set before on exit.
"""
import contextlib
import ctypes

from ._lib import check, lib


def tune_set(name, value):
    check(lib().mi_tune_set(name.encode(), int(value)))


def tune_clear(name=None):
    check(lib().mi_tune_clear(name.encode() if name is not None else None))


def tune_get(name):
    """The switch's value, or None while it holds its default."""
    v, s = ctypes.c_int64(0), ctypes.c_int(0)
    check(lib().mi_tune_get(name.encode(), ctypes.byref(v), ctypes.byref(s)))
    return v.value if s.value else None


@contextlib.contextmanager
def tuned(**knobs):
    """Set switches for the duration of a block (None clears one); the previous values come back afterwards."""
    before = {k: tune_get(k) for k in knobs}
    try:
        for k, v in knobs.items():
            if v is None:
                tune_clear(k)
            else:
                tune_set(k, v)
        yield
    finally:
        for k, v in before.items():
            if v is None:
                tune_clear(k)
            else:
                tune_set(k, v)
