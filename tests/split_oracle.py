"""Oracle-side shares of the single-proof latency mode (TEST INFRASTRUCTURE; checker only).

Restates what mi_groth16_prove_share computes, with the oracle's CPU MSMs: rank k of `world` takes
the contiguous slice [n k / world, n (k + 1) / world) of every query -- h (the first d - 1 positions of
the bit-reversed coefficient order the device keeps H and h in; position d - 1 is coefficient d - 1,
the one bellman drops), l (aux), a (inputs, then aux in A's column density) and b_g1 / b_g2
(inputs and aux in B's density; bellman's a/b density, oracle.cpp or_groth16_prove) -- and encodes
the five sums H | L | A | B_G1 | B_G2 in zcash uncompressed form (576 bytes).
"""
import numpy as np

SHARE_BYTES = 576
G1_INF = bytes([0x40]) + bytes(95)
G2_INF = bytes([0x40]) + bytes(191)


def densities(n_in, n_aux, mats):
    """-> (idx_a, idx_b): variable indices whose z value scales each a / b_g1 / b_g2 point."""
    used = []
    for m in (0, 1):
        _, col, _ = mats[m]
        used.append(set(int(v) for v in col))
    idx_a = list(range(n_in)) + [v for v in range(n_in, n_in + n_aux) if v in used[0]]
    idx_b = [v for v in range(n_in + n_aux) if v in used[1]]
    return idx_a, idx_b


def _slice(n, rank, world):
    return n * rank // world, n * (rank + 1) // world


def shares(oracle, params, n_in, n_aux, mats, z: bytes, world: int):
    """The `world` oracle shares of one proof (list of 576-byte records, rank order)."""
    ex = params.export()
    _, _, hb = params.prove(z, 0, 0, want_h=True)
    idx_a, idx_b = densities(n_in, n_aux, mats)
    zs = np.frombuffer(z, dtype=np.uint8).reshape(-1, 32)

    def msm(bases, esz, scal, lo, hi, g2=False):
        if hi == lo:
            return G2_INF if g2 else G1_INF
        fn = oracle.msm_g2 if g2 else oracle.msm_g1
        return fn(bases[esz * lo:esz * hi], scal[32 * lo:32 * hi])

    zaux = zs[n_in:].tobytes()
    za = zs[idx_a].tobytes()
    zb = zs[idx_b].tobytes()
    log_d = params.d.bit_length() - 1
    rev = [int(format(i, f"0{log_d}b")[::-1], 2) for i in range(params.d - 1)] if log_d else []
    hq = np.frombuffer(ex["h"], dtype=np.uint8).reshape(-1, 96)
    hc = np.frombuffer(hb, dtype=np.uint8).reshape(-1, 32)
    h_perm, hb_perm = hq[rev].tobytes(), hc[rev].tobytes()
    out = []
    for k in range(world):
        rec = msm(h_perm, 96, hb_perm, *_slice(params.d - 1, k, world))
        rec += msm(ex["l"], 96, zaux, *_slice(n_aux, k, world))
        rec += msm(ex["a"], 96, za, *_slice(len(idx_a), k, world))
        lo, hi = _slice(len(idx_b), k, world)
        rec += msm(ex["b_g1"], 96, zb, lo, hi) + msm(ex["b_g2"], 192, zb, lo, hi, g2=True)
        assert len(rec) == SHARE_BYTES
        out.append(rec)
    return out


def h_coeffs_perm(params, z: bytes) -> bytes:
    """The d H coefficients in the device's bit-reversed h order (what mi_groth16_h_coeffs_dev writes): the d - 1
    coefficients bellman keeps at positions bitrev(i), the last position (coefficient d - 1) zero."""
    _, _, hb = params.prove(z, 0, 0, want_h=True)
    log_d = params.d.bit_length() - 1
    hc = np.frombuffer(hb, dtype=np.uint8).reshape(-1, 32)
    out = np.zeros((params.d, 32), dtype=np.uint8)
    for i in range(params.d - 1):
        out[int(format(i, f"0{log_d}b")[::-1], 2) if log_d else 0] = hc[i]
    return out.tobytes()


def shares_ranges(oracle, params, n_in, n_aux, mats, z: bytes, ranges_list, h_perm_coeffs: bytes = None):
    """Oracle shares over explicit query ranges (what mi_groth16_prove_share_ranges computes): one
    [(first, count)] x 4 list (H in the bit-reversed h order, L, A, B) per share.  h_perm_coeffs: H coefficients
    received from elsewhere (h_coeffs_perm's layout), used instead of the oracle's own (the H-split protocol)."""
    ex = params.export()
    _, _, hb = params.prove(z, 0, 0, want_h=True)
    idx_a, idx_b = densities(n_in, n_aux, mats)
    zs = np.frombuffer(z, dtype=np.uint8).reshape(-1, 32)

    def msm(bases, esz, scal, lo, cnt, g2=False):
        if cnt == 0:
            return G2_INF if g2 else G1_INF
        fn = oracle.msm_g2 if g2 else oracle.msm_g1
        return fn(bases[esz * lo:esz * (lo + cnt)], scal[32 * lo:32 * (lo + cnt)])

    zaux, za, zb = zs[n_in:].tobytes(), zs[idx_a].tobytes(), zs[idx_b].tobytes()
    log_d = params.d.bit_length() - 1
    rev = [int(format(i, f"0{log_d}b")[::-1], 2) for i in range(params.d - 1)] if log_d else []
    hq = np.frombuffer(ex["h"], dtype=np.uint8).reshape(-1, 96)
    hc = np.frombuffer(hb, dtype=np.uint8).reshape(-1, 32)
    h_perm, hb_perm = hq[rev].tobytes(), hc[rev].tobytes()
    if h_perm_coeffs is not None:
        hb_perm = h_perm_coeffs[:32 * (params.d - 1)]
    out = []
    for (h, l, a, b) in ranges_list:
        rec = msm(h_perm, 96, hb_perm, *h) + msm(ex["l"], 96, zaux, *l) + msm(ex["a"], 96, za, *a)
        rec += msm(ex["b_g1"], 96, zb, *b) + msm(ex["b_g2"], 192, zb, *b, g2=True)
        assert len(rec) == SHARE_BYTES
        out.append(rec)
    return out
