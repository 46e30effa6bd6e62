"""Generate the committed golden fixtures from the independent pure-Python restatement (pyref.py).

    python tests/golden/gen_golden.py            # writes tests/golden/*.json

The reference (NilFoundation/crypto3-fil-proofs) holds no golden vector for this path and its
crypto3 submodules are empty, so the fixtures pin:
  * published BLS12-381 constants (generator compressed encodings, group order, 2-adic root),
  * the pure-Python restatement's outputs for NTT / MSM / Groth16 on seeded inputs,
  * a pairing-equation verification of every Groth16 fixture proof (pure Python).
If the C++ oracle is built, the script also asserts the oracle reproduces every vector.
"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import circuits  # noqa: E402
import pyref as py  # noqa: E402

# Published constants (zcash/IETF BLS12-381 serialization of the standard generators)
G1_GEN_COMPRESSED = ("97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1a"
                     "effb3af00adb22c6bb")
G2_GEN_COMPRESSED = ("93e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d"
                     "57e5ac7d055d042b7e024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3"
                     "d1770bac0326a805bbefd48056c8c121bdb8")
# bellman/zkcrypto Fr::ROOT_OF_UNITY (= 7^((r-1)/2^32))
FR_ROOT_OF_UNITY = 0x16A2A19EDFE81F20D09B681922C813B4B63683508C2280B93829971F439F0D2B


def hx(b):
    return b.hex()


def field_kat():
    assert py.g1_compressed(py.G1).hex() == G1_GEN_COMPRESSED
    assert py.g2_compressed(py.G2).hex() == G2_GEN_COMPRESSED
    assert py.ROOT_OF_UNITY == FR_ROOT_OF_UNITY
    assert py.E1.on_curve(py.G1) and py.E2.on_curve(py.G2)
    assert py.E1.mul(py.E1.from_aff(py.G1), py.R - 1) is not None
    assert py.E1.add(py.E1.mul(py.E1.from_aff(py.G1), py.R - 1), py.E1.from_aff(py.G1)) is None
    rng = py.SplitMix64(3)
    frs = [rng.fr() for _ in range(8)]
    return dict(
        g1_generator_uncompressed=hx(py.g1_uncompressed(py.G1)),
        g2_generator_uncompressed=hx(py.g2_uncompressed(py.G2)),
        g1_generator_compressed=G1_GEN_COMPRESSED,
        g2_generator_compressed=G2_GEN_COMPRESSED,
        roots_of_unity={str(k): hx(py.fr_le(py.omega(k))) for k in (1, 2, 10, 20, 26, 27, 32)},
        fr_mul=[[hx(py.fr_le(a)), hx(py.fr_le(b)), hx(py.fr_le(a * b))] for a, b in zip(frs[::2], frs[1::2])],
        fr_inv=[[hx(py.fr_le(a)), hx(py.fr_le(pow(a, py.R - 2, py.R)))] for a in frs],
    )


def ntt_vectors():
    out = {}
    for log_n, seed in ((1, 9), (3, 9), (6, 9)):
        rng = py.SplitMix64(seed)
        a = [rng.fr() for _ in range(1 << log_n)]
        ent = {"input": hx(b"".join(py.fr_le(x) for x in a))}
        for kind, name in enumerate(("fft", "ifft", "coset_fft", "icoset_fft")):
            ent[name] = hx(b"".join(py.fr_le(x) for x in py.domain(a, log_n, kind)))
        out[str(log_n)] = ent
    return out


def msm_vectors():
    out = {}
    for name, curve, gen, n, enc in (("g1", py.E1, py.g1_mul_gen, 64, py.g1_uncompressed),
                                     ("g2", py.E2, py.g2_mul_gen, 16, py.g2_uncompressed)):
        rk = py.SplitMix64(42)
        rs = py.SplitMix64(7)
        ks = [rk.fr() for _ in range(n)]
        bases = [gen(k) for k in ks]
        scalars = [rs.fr() for _ in range(n)]
        # edge scalars: 0, 1, r-1, 2, a repeated base
        scalars[0], scalars[1], scalars[2], scalars[3] = 0, 1, py.R - 1, 2
        bases[5] = bases[4]
        res = py.msm(curve, bases, scalars)
        # size-independent identity: MSM over k_i G equals (sum s_i k_i) G
        ks[5] = ks[4]
        assert res == gen(sum(s * k for s, k in zip(scalars, ks)) % py.R)
        out[name] = dict(bases=hx(b"".join(enc(b) for b in bases)),
                         scalars=hx(b"".join(py.fr_le(s) for s in scalars)),
                         result=hx(enc(res)))
    return out


def groth16_vector(name, n_in, n_aux, rows, z):
    circ = py.Circuit(n_in, n_aux, rows)
    assert circ.satisfied(z)
    tox = circuits.toxic()
    r, s = circuits.blinding()
    t0 = time.time()
    pk = py.keygen(circ, tox)
    proof, raw, h = py.prove(pk, circ, z, r, s)
    ok = py.verify(pk, z[:n_in], raw)
    assert ok, "pairing check failed for " + name
    print(f"  {name}: d={pk['d']} rows={len(rows)} vars={n_in + n_aux} keygen+prove+verify {time.time() - t0:.1f}s")
    return dict(
        num_inputs=n_in, num_aux=n_aux, num_constraints=len(rows), d=pk["d"],
        toxic=[hx(py.fr_le(t)) for t in tox], r=hx(py.fr_le(r)), s=hx(py.fr_le(s)),
        proof=hx(proof), raw=hx(raw),
        h_sha256=hashlib.sha256(b"".join(py.fr_le(x) for x in h)).hexdigest(),
        query_sizes=[len(pk["h"]), len(pk["l"]), len(pk["a"]), len(pk["b_g1"]), len(pk["b_g2"])],
        vk_alpha_g1=hx(py.g1_uncompressed(pk["alpha_g1"])),
        pairing_verified=ok,
    )


def main():
    t0 = time.time()
    fx = {}
    fx["field"] = field_kat()
    fx["ntt"] = ntt_vectors()
    fx["msm"] = msm_vectors()
    print("kat/ntt/msm done %.1fs" % (time.time() - t0))
    g = {}
    for seed, rows in ((11, 24), (12, 60)):
        n_in, n_aux, rws, z = circuits.random_circuit(seed, rows)
        g["random_%d_%d" % (seed, rows)] = groth16_vector("random_%d_%d" % (seed, rows), n_in, n_aux, rws, z)
    n_in, n_aux, rws, z = circuits.toy_chain(1022)
    g["toy_chain_1022"] = groth16_vector("toy_chain_1022", n_in, n_aux, rws, z)
    fx["groth16"] = g
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(fx, f, indent=1, sort_keys=True)
    print("wrote golden.json in %.1fs" % (time.time() - t0))


if __name__ == "__main__":
    main()
