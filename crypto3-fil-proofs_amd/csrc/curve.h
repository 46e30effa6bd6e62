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

// Endomorphism membership tests (the checked key load's kernel, round 6): ~70 group operations per point instead of
// the ~384 of r P, the tests of Scott, "A note on group membership tests for G1, G2 and GT on BLS pairing-friendly
// curves" (eprint 2021/1130, proof of correctness eprint 2022/352), as zkcrypto's bls12_381 is_torsion_free runs them:
//   G1: sigma(P) == -[z^2] P,  sigma(x, y) = (beta^2 x, y), beta^2 the cube root of unity acting as -z^2 on G1 (the
//       other root, glv.h's beta, acts as z^2 - 1);
//   G2: psi(P) == [z] P,  psi(x, y) = (conj(x) cx, conj(y) cy), cx = (1 + u)^-((p - 1) / 3), cy = (1 + u)^-((p - 1) / 2)
// with z = -0xd201000000010000.  tests/host/grouplaw_check.cpp compares both with r P == O on subgroup points, on
// the non-subgroup points of the GPU tests and on cofactor-torsion and mixed points; the constants were derived and
// the tests checked the same way over Python integers first.
constexpr uint64_t BLS_Z_ABS = 0xd201000000010000ull;
// canonical little-endian words: beta^2, cx (c0 = 0), cy
constexpr uint32_t SUBGROUP_BETA2_RAW[12] = {0xfffefffeu, 0x2e01ffffu, 0x620a0002u, 0xde17d813u, 0xe6f89688u,
                                             0xddb3a93bu, 0x6a0f77eau, 0xba69c607u, 0xdf76ce51u, 0x5f19672fu,
                                             0x00000000u, 0x00000000u};
constexpr uint32_t SUBGROUP_CX1_RAW[12] = {0x0000aaadu, 0x8bfd0000u, 0x4f49fffdu, 0x409427ebu, 0x0fb85f9bu,
                                           0x897d2965u, 0x89759ad4u, 0xaa0d857du, 0x63d4de85u, 0xec024086u,
                                           0x397fe699u, 0x1a0111eau};
constexpr uint32_t SUBGROUP_CY0_RAW[12] = {0x121bdea2u, 0xf1ee7b04u, 0x3e67fa0au, 0x304466cfu, 0xf61eb45eu,
                                           0xef396489u, 0x30b1cf60u, 0x1c3dedd9u, 0xd77a2cd9u, 0xe2e9c448u,
                                           0x0180a68eu, 0x135203e6u};
constexpr uint32_t SUBGROUP_CY1_RAW[12] = {0xede3cc09u, 0xc81084fbu, 0x72ec05f4u, 0xee67992fu, 0x009241c5u,
                                           0x77f76e17u, 0xc2d3435eu, 0x48395dabu, 0x6bd17ffeu, 0x6831e36du,
                                           0x37ff400bu, 0x06af0e04u};
struct SubgroupConsts {
    fq_t beta2;
    fq2_t cx, cy;
};
inline SubgroupConsts subgroup_consts() {  // host: the Montgomery images, passed to the kernel
    auto fq = [](const uint32_t *w) {
        fq32_t raw;
        for (int i = 0; i < 12; i++) raw.v[i] = w[i];
        return fq_from_raw(raw);
    };
    SubgroupConsts s;
    s.beta2 = fq(SUBGROUP_BETA2_RAW);
    s.cx = {fq_t::zero(), fq(SUBGROUP_CX1_RAW)};
    s.cy = {fq(SUBGROUP_CY0_RAW), fq(SUBGROUP_CY1_RAW)};
    return s;
}
// [|z|] q by double-and-add over the 6 set bits of |z| (64 doublings)
template <class F>
MI_HD XYZZ<F> xyzz_mul_zabs_inl(const XYZZ<F> &q) {
    XYZZ<F> r = q;  // bit 63
#pragma unroll 1
    for (int b = 62; b >= 0; b--) {
        r = xyzz_dbl_inl(r);
        if ((BLS_Z_ABS >> b) & 1) r = xyzz_add_inl(r, q);
    }
    return r;
}
// XYZZ q equals the affine (x, y): X = x ZZ and Y = y ZZZ (q finite)
template <class F>
MI_HD bool xyzz_eq_affine(const XYZZ<F> &q, const F &x, const F &y) {
    return !q.is_inf() && q.X == x * q.ZZ && q.Y == y * q.ZZZ;
}
MI_HD bool in_prime_subgroup_fast(const Affine<fq_t> &a, const SubgroupConsts &s) {
    if (a.is_inf()) return true;
    const XYZZ<fq_t> z2 = xyzz_mul_zabs_inl(xyzz_mul_zabs_inl(xyzz_from_affine(a)));  // [z^2] P
    return xyzz_eq_affine(z2, s.beta2 * a.x, -a.y);                                  // == -sigma(P)
}
MI_HD bool in_prime_subgroup_fast(const Affine<fq2_t> &a, const SubgroupConsts &s) {
    if (a.is_inf()) return true;
    const XYZZ<fq2_t> q = xyzz_mul_zabs_inl(xyzz_from_affine(a));  // [|z|] P = -[z] P
    const fq2_t px = fq2_t{a.x.c0, -a.x.c1} * s.cx, py = fq2_t{a.y.c0, -a.y.c1} * s.cy;
    return xyzz_eq_affine(q, px, -py);  // -[z] P == -psi(P)
}

}  // namespace mi
