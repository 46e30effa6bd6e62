"""Test helper: BLS12-381 points that ARE on the curve but NOT in the prime-order subgroup (TEST
INFRASTRUCTURE).  bellman's checked Parameters::read (from_uncompressed) must refuse them; the
unchecked read (from_uncompressed_unchecked) accepts them.  Pure Python over pyref's fields."""
from pyref import E1, E2, P, R, g1_uncompressed, g2_uncompressed


def _in_subgroup(E, a):
    """r a == O, as (r - 1) a + a (pyref's Curve.mul reduces its scalar mod r)."""
    pa = E.from_aff(a)
    return E.add(E.mul(pa, R - 1), pa) is None


def _fq_sqrt(a):
    y = pow(a, (P + 1) // 4, P)  # p = 3 mod 4
    return y if y * y % P == a % P else None


def _fq2_sqrt(a):
    """sqrt in Fq[u]/(u^2 + 1) by the norm method: y0^2 = (a0 +- |a|) / 2, y1 = a1 / (2 y0)."""
    a0, a1 = a
    n = _fq_sqrt((a0 * a0 + a1 * a1) % P)
    if n is None:
        return None
    inv2 = pow(2, P - 2, P)
    for t in ((a0 + n) * inv2 % P, (a0 - n) * inv2 % P):
        y0 = _fq_sqrt(t)
        if y0 is None or y0 == 0:
            continue
        y1 = a1 * pow(2 * y0, P - 2, P) % P
        if ((y0 * y0 - y1 * y1) % P, 2 * y0 * y1 % P) == (a0 % P, a1 % P):
            return (y0, y1)
    return None


def g1_non_subgroup(start=5):
    """(affine point, uncompressed bytes): on y^2 = x^3 + 4, r P != O."""
    x = start
    while True:
        y = _fq_sqrt((x * x * x + 4) % P)
        if y is not None:
            a = (x, y)
            assert E1.on_curve(a)
            if not _in_subgroup(E1, a):
                return a, g1_uncompressed(a)
        x += 1


def g2_non_subgroup(start=3):
    """(affine point, uncompressed bytes): on the twist y^2 = x^3 + 4(u + 1), r P != O."""
    k = start
    while True:
        x = (k, 1)
        x3 = E2.F.mul(E2.F.mul(x, x), x)
        y = _fq2_sqrt(E2.F.add(x3, (4, 4)))
        if y is not None:
            a = (x, y)
            assert E2.on_curve(a)
            if not _in_subgroup(E2, a):
                return a, g2_uncompressed(a)
        k += 1
