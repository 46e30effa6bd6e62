"""CPU: the device group law (csrc/field.h + csrc/curve.h, the code k_accum_level0 and the bucket
reduction inline) compiled for the host under AddressSanitizer + UndefinedBehaviorSanitizer and checked
against the oracle's G1/G2 group law (tests/host/grouplaw_check.cpp).

Covers the lazily reduced intermediates of the XYZZ additions (unreduced subtractions feeding
multiplications, the one-pass X3) on random and extreme (near 2p) values, every branch of the mixed and
full additions (doubling, P + (-P), infinity operands, both representatives v and v + p of each
coordinate, negated signed-digit points), and the host-side G2 path.  No GPU is used."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.fixture(scope="module")
def grouplaw_bin(oracle):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out_dir = os.path.join(ROOT, "tests", "host", "build")
    os.makedirs(out_dir, exist_ok=True)
    exe = os.path.join(out_dir, "grouplaw_check")
    lib_dir = os.path.join(ROOT, "oracle", "build")  # liboracle.so (built by the oracle fixture)
    # -O0: the fully unrolled limb code takes minutes to instrument at -O1 and the checks do not need it
    cmd = [HIPCC, "-x", "hip", "--offload-host-only", "-std=c++17", "-O0",
           "-fno-gpu-sanitize", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-I", os.path.join(ROOT, "crypto3-fil-proofs_amd", "csrc"),
           "-I", os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "host", "grouplaw_check.cpp"),
           "-L", lib_dir, "-loracle", "-Wl,-rpath," + lib_dir, "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    yield exe
    shutil.rmtree(out_dir, ignore_errors=True)


def test_device_group_law_on_host_under_sanitizers(grouplaw_bin):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([grouplaw_bin], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "grouplaw OK" in r.stdout
