// curve.h -- BLS12-381 G1 (over Fq) and G2 (over Fq2) group law for the MSM hot loop.
//
// Restates crypto3 algebra's curve arithmetic ([NOT IN TREE]: libs/crypto/algebra, g1_type /
// g2_type of bls12<381>, core/crypto/scheme_params.hpp:40-41).  Buckets use XYZZ coordinates
// (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2): a mixed add costs 8M + 2S with no field inversion and no
// doubling of Z, which is what the bucket loop does ~N * windows times.
// Affine infinity is encoded as (0, 0) (not on the curve: 0 != 0 + b).
#pragma once
#include "field.h"

namespace mi {

// Stored G1 bases are gathered at random by the bucket accumulation, one record per mixed addition. A
// 112-byte record straddles two 128-byte lines for 7 of 8 records; padded to an aligned 128 bytes every
// gather fetches one line.  The gathered bytes cost power, not cycles: the accumulation's cycles per
// addition are unchanged, but the core clock under load rises from 2.08 to 2.18 GHz, +6 % mixed additions
// per second (microbench/maddloop.hip, profiles/r03_maddloop2.jsonl).  G2 records stay 224 bytes: an
// aligned 256-byte form measured no gain for the lane-pair addition (1.73 vs 1.71 G madd/s,
// profiles/r03_maddloop3.jsonl), whose VALU work per gathered byte is 3x G1's, and would cost the 32 GiB
// Window-PoSt key 2 GB.  In registers the padding does not exist.
template <class F>
struct AffineAlign {
    static constexpr size_t value = 16;
};
template <>
struct AffineAlign<fq_t> {
    static constexpr size_t value = 128;
};

// Infinity tests.  An affine infinity is stored as raw (0, 0) and an XYZZ infinity has ZZ = 0; Fq coordinates
// that are zero mod p are zero as limbs there (every ZZ is a Montgomery product, |product| < p, or a constant),
// so Fq tests the limbs (no modular check); other coordinate types use their is_zero.
template <class F>
MI_HD bool coord_zero(const F &a) { return a.is_zero(); }
MI_HD bool coord_zero(const fq_t &a) { return a.is_raw_zero(); }

template <class F>
struct alignas(AffineAlign<F>::value) Affine {
    F x, y;
    MI_HD bool is_inf() const { return coord_zero(x) && coord_zero(y); }
    MI_HD static Affine inf() { return {F::zero(), F::zero()}; }
};

template <class F>
struct alignas(16) XYZZ {
    F X, Y, ZZ, ZZZ;
    MI_HD static XYZZ inf() { return {F::one(), F::one(), F::zero(), F::zero()}; }
    MI_HD bool is_inf() const { return coord_zero(ZZ); }
};

template <class F>
MI_HD XYZZ<F> xyzz_from_affine(const Affine<F> &a) {
    if (a.is_inf()) return XYZZ<F>::inf();
    return {a.x, a.y, F::one(), F::one()};
}

template <class F>
MI_HD Affine<F> affine_neg(const Affine<F> &a) {
    return {a.x, -a.y};
}

template <class F>
MI_HD XYZZ<F> xyzz_neg(const XYZZ<F> &p) {
    return {p.X, -p.Y, p.ZZ, p.ZZZ};
}

// dbl-2008-s-1 (a = 0)
template <class F>
MI_HD XYZZ<F> xyzz_dbl_inl(const XYZZ<F> &p) {
    if (p.is_inf()) return p;
    F U = dbl(p.Y);
    F V = sqr(U);
    F W = U * V;
    F S = p.X * V;
    F X2 = sqr(p.X);
    F M = X2 + dbl(X2);
    XYZZ<F> r;
    r.X = sqr(M) - dbl(S);
    r.Y = M * (S - r.X) - W * p.Y;
    r.ZZ = V * p.ZZ;
    r.ZZZ = W * p.ZZZ;
    return r;
}
template <class F>
MI_NOINL XYZZ<F> xyzz_dbl(const XYZZ<F> &p) {
    return xyzz_dbl_inl(p);
}

// mdbl-2008-s-1: double an affine point
template <class F>
MI_HD XYZZ<F> xyzz_dbl_affine_inl(const Affine<F> &a) {
    F U = dbl(a.y);
    F V = sqr(U);
    F W = U * V;
    F S = a.x * V;
    F X2 = sqr(a.x);
    F M = X2 + dbl(X2);
    XYZZ<F> r;
    r.X = sqr(M) - dbl(S);
    r.Y = M * (S - r.X) - W * a.y;
    r.ZZ = V;
    r.ZZZ = W;
    return r;
}
template <class F>
MI_NOINL XYZZ<F> xyzz_dbl_affine(const Affine<F> &a) {
    return xyzz_dbl_affine_inl(a);
}

// Lazy-reduction hooks of the additions (field.h "lazy forms"): Fq takes the unreduced forms, every
// other coordinate type (Fq2, the G2 lane-pair halves) the plain reduced operators.
template <class F>
MI_HD F lazy_sub(const F &a, const F &b) { return a - b; }
template <class F>
MI_HD F lazy_neg(const F &a) { return -a; }
template <class F>
MI_HD F x3_of(const F &r2, const F &ppp, const F &q) { return r2 - ppp - dbl(q); }
MI_HD fq_t lazy_sub(const fq_t &a, const fq_t &b) { return fq_sub_lazy(a, b); }
MI_HD fq_t lazy_neg(const fq_t &a) { return fq_neg_lazy(a); }
MI_HD fq_t x3_of(const fq_t &r2, const fq_t &ppp, const fq_t &q) { return fq_x3(r2, ppp, q); }

// *_inl: force-inlined bodies for the hot kernels (no call ABI, no scratch); the plain names
// are noinline wrappers for cold code (host assembly, table builds, reductions).

// madd-2008-s: p (XYZZ) + q (affine, may be infinity)
template <class F>
MI_HD XYZZ<F> xyzz_add_affine_inl(const XYZZ<F> &p, const Affine<F> &q) {
    if (q.is_inf()) return p;
    if (p.is_inf()) return xyzz_from_affine(q);
    F U2 = q.x * p.ZZ;
    F S2 = q.y * p.ZZZ;
    F P = U2 - p.X;
    F R = S2 - p.Y;
    if (P.is_zero()) {
        if (R.is_zero()) return xyzz_dbl_affine_inl(q);
        return XYZZ<F>::inf();
    }
    F PP = sqr(P);
    F PPP = P * PP;
    F Q = p.X * PP;
    XYZZ<F> r;
    r.X = x3_of(sqr(R), PPP, Q);
    r.Y = mul_add(R, lazy_sub(Q, r.X), lazy_neg(p.Y), PPP);  // R (Q - X3) - Y1 PPP, one reduction
    r.ZZ = p.ZZ * PP;
    r.ZZZ = p.ZZZ * PPP;
    return r;
}
template <class F>
MI_NOINL XYZZ<F> xyzz_add_affine(const XYZZ<F> &p, const Affine<F> &q) {
    return xyzz_add_affine_inl(p, q);
}

// add-2008-s: p + q, both XYZZ
template <class F>
MI_HD XYZZ<F> xyzz_add_inl(const XYZZ<F> &p, const XYZZ<F> &q) {
    if (q.is_inf()) return p;
    if (p.is_inf()) return q;
    F U1 = p.X * q.ZZ;
    F U2 = q.X * p.ZZ;
    F S1 = p.Y * q.ZZZ;
    F S2 = q.Y * p.ZZZ;
    F P = U2 - U1;
    F R = S2 - S1;
    if (P.is_zero()) {
        if (R.is_zero()) return xyzz_dbl_inl(p);
        return XYZZ<F>::inf();
    }
    F PP = sqr(P);
    F PPP = P * PP;
    F Q = U1 * PP;
    XYZZ<F> r;
    r.X = x3_of(sqr(R), PPP, Q);
    r.Y = mul_add(R, lazy_sub(Q, r.X), lazy_neg(S1), PPP);
    r.ZZ = p.ZZ * q.ZZ * PP;
    r.ZZZ = p.ZZZ * q.ZZZ * PPP;
    return r;
}
template <class F>
MI_NOINL XYZZ<F> xyzz_add(const XYZZ<F> &p, const XYZZ<F> &q) {
    return xyzz_add_inl(p, q);
}

// XYZZ -> affine (one inversion)
template <class F>
MI_HD Affine<F> xyzz_to_affine_inl(const XYZZ<F> &p) {
    if (p.is_inf()) return Affine<F>::inf();
    F izzz = inverse_inl(p.ZZZ);
    F izz_sq = sqr(p.ZZ * izzz);  // (ZZ/ZZZ)^2 = 1/ZZ  (ZZ^3 = ZZZ^2)
    return {p.X * izz_sq, p.Y * izzz};
}
template <class F>
MI_NOINL Affine<F> xyzz_to_affine(const XYZZ<F> &p) {
    return xyzz_to_affine_inl(p);
}

// scalar multiplication by a canonical little-endian word scalar
template <class F>
MI_HD XYZZ<F> xyzz_mul_inl(const XYZZ<F> &p, const uint32_t *k, int nwords) {
    XYZZ<F> r = XYZZ<F>::inf();
#pragma unroll 1
    for (int i = nwords - 1; i >= 0; i--)
#pragma unroll 1
        for (int b = 31; b >= 0; b--) {
            r = xyzz_dbl_inl(r);
            if ((k[i] >> b) & 1) r = xyzz_add_inl(r, p);
        }
    return r;
}
template <class F>
MI_NOINL XYZZ<F> xyzz_mul(const XYZZ<F> &p, const uint32_t *k, int nwords) {
    return xyzz_mul_inl(p, k, nwords);
}

typedef Affine<fq_t> g1_affine_t;
typedef Affine<fq2_t> g2_affine_t;
typedef XYZZ<fq_t> g1_xyzz_t;
typedef XYZZ<fq2_t> g2_xyzz_t;

// y^2 = x^3 + 4 (G1) and y^2 = x^3 + 4 (u + 1) (G2); the affine infinity (0, 0) is not on the curve,
// callers handle it by its flag
MI_HD bool g1_on_curve(const g1_affine_t &a) { return sqr(a.y) == sqr(a.x) * a.x + fq_small(4); }
MI_HD bool g2_on_curve(const g2_affine_t &a) {
    const fq2_t b = {fq_small(4), fq_small(4)};
    return sqr(a.y) == sqr(a.x) * a.x + b;
}
// r * a == O: membership in the prime-order subgroup, the check zcash/bellman's checked
// from_uncompressed adds to the curve equation (Parameters::read with checked = true)
template <class F>
MI_HD bool in_prime_subgroup(const Affine<F> &a) {
    if (a.is_inf()) return true;
    uint32_t r[8];
    MI_UNROLL for (int i = 0; i < 8; i++) r[i] = FrDesc::MOD[i];
    return xyzz_mul_inl(xyzz_from_affine(a), r, 8).is_inf();
}

}  // namespace mi
