"""GPU: the C++ host layer (include/mi355x_groth16.hpp, examples/prove_synthetic.cpp) produces the
same proofs as the Python binding for the same synthetic circuit, key and blinding."""
import os
import subprocess

import pytest

import fil_groth16 as fg
from fil_groth16 import synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_circuit_proofs_match_python(ctx):
    pkg = os.path.join(ROOT, "crypto3-fil-proofs_amd")
    exe = os.path.join(pkg, "build", "prove_synthetic")
    if not os.path.exists(exe):  # build() makes it; objects do not travel to the GPU box, so link directly
        subprocess.check_call(["g++", "-std=c++17", "-O2", "-I" + os.path.join(ROOT, "include"),
                               os.path.join(pkg, "examples", "prove_synthetic.cpp"), "-L" + os.path.join(pkg, "build"),
                               "-lfilgpu", "-Wl,-rpath,$ORIGIN", "-o", exe], timeout=120)
    out = subprocess.run([os.path.join(pkg, "build", "prove_synthetic"), "10", "3"], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    cpp = [bytes.fromhex(l) for l in out.stdout.split()]
    sc = synth.SynthCircuit(10, 4, 1)
    gc = sc.load(ctx)
    pk = fg.generate_random_parameters(ctx, gc, [11, 12, 13, 14, 15])
    py = [fg.prove(ctx, pk, gc, sc.z_bytes(), 100 + k, 200 + k) for k in range(3)]
    assert cpp == py
