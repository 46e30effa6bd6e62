// oracle.cpp -- CPU restatement of the BLS12-381 Groth16 hot path.
// TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline.
// Parity unpinned against the reference itself (unbuildable, no golden vectors); pinned by published
// constants, the independent Python restatement and pairing checks -- see oracle.h / DESIGN.md §3.
// The product (libfilgpu.so) never links or calls this file.  See oracle.h for the reference map.
//
// Style is intentionally different from the device code: 64-bit limbs with unsigned __int128
// products (the device uses 32-bit limbs and v_mad_u64_u32), Jacobian coordinates (the device
// uses XYZZ buckets), bellman's serial radix-2 FFT (the device uses a multi-pass LDS NTT) and
// a per-thread-chunk unsigned-window Pippenger (the device uses signed digits + sorted buckets).
#include "oracle.h"

#include <omp.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

typedef unsigned __int128 u128;

namespace {

// ------------------------------------------------------------------------------------------
// Montgomery field over N 64-bit limbs
// ------------------------------------------------------------------------------------------
struct FqTag {};
struct FrTag {};

template <typename Tag, int N>
struct Fp {
    uint64_t l[N];
};

template <typename Tag, int N>
struct Consts {
    static const uint64_t MOD[N];
    static const uint64_t R[N];
    static const uint64_t R2[N];
    static const uint64_t INV;
};

template <>
const uint64_t Consts<FqTag, 6>::MOD[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                                           0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
template <>
const uint64_t Consts<FqTag, 6>::R[6] = {0x760900000002fffdULL, 0xebf4000bc40c0002ULL, 0x5f48985753c758baULL,
                                         0x77ce585370525745ULL, 0x5c071a97a256ec6dULL, 0x15f65ec3fa80e493ULL};
template <>
const uint64_t Consts<FqTag, 6>::R2[6] = {0xf4df1f341c341746ULL, 0x0a76e6a609d104f1ULL, 0x8de5476c4c95b6d5ULL,
                                          0x67eb88a9939d83c0ULL, 0x9a793e85b519952dULL, 0x11988fe592cae3aaULL};
template <>
const uint64_t Consts<FqTag, 6>::INV = 0x89f3fffcfffcfffdULL;

template <>
const uint64_t Consts<FrTag, 4>::MOD[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL,
                                           0x73eda753299d7d48ULL};
template <>
const uint64_t Consts<FrTag, 4>::R[4] = {0x00000001fffffffeULL, 0x5884b7fa00034802ULL, 0x998c4fefecbc4ff5ULL,
                                         0x1824b159acc5056fULL};
template <>
const uint64_t Consts<FrTag, 4>::R2[4] = {0xc999e990f3f29c6dULL, 0x2b6cedcb87925c23ULL, 0x05d314967254398fULL,
                                          0x0748d9d99f59ff11ULL};
template <>
const uint64_t Consts<FrTag, 4>::INV = 0xfffffffeffffffffULL;

template <typename Tag, int N>
struct F {
    typedef Fp<Tag, N> T;
    typedef Consts<Tag, N> C;

    static T zero() {
        T r;
        memset(r.l, 0, sizeof r.l);
        return r;
    }
    static T one() {
        T r;
        memcpy(r.l, C::R, sizeof r.l);
        return r;
    }
    static bool is_zero(const T &a) {
        uint64_t x = 0;
        for (int i = 0; i < N; i++) x |= a.l[i];
        return x == 0;
    }
    static bool eq(const T &a, const T &b) { return memcmp(a.l, b.l, sizeof a.l) == 0; }
    // a >= b on raw limbs
    static bool geq(const uint64_t *a, const uint64_t *b) {
        for (int i = N - 1; i >= 0; i--) {
            if (a[i] != b[i]) return a[i] > b[i];
        }
        return true;
    }
    static void sub_raw(uint64_t *r, const uint64_t *a, const uint64_t *b) {
        uint64_t borrow = 0;
        for (int i = 0; i < N; i++) {
            u128 d = (u128)a[i] - b[i] - borrow;
            r[i] = (uint64_t)d;
            borrow = (uint64_t)(d >> 64) & 1;
        }
    }
    static T add(const T &a, const T &b) {
        T r;
        uint64_t carry = 0;
        for (int i = 0; i < N; i++) {
            u128 s = (u128)a.l[i] + b.l[i] + carry;
            r.l[i] = (uint64_t)s;
            carry = (uint64_t)(s >> 64);
        }
        if (carry || geq(r.l, C::MOD)) sub_raw(r.l, r.l, C::MOD);
        return r;
    }
    static T sub(const T &a, const T &b) {
        T r;
        uint64_t borrow = 0;
        for (int i = 0; i < N; i++) {
            u128 d = (u128)a.l[i] - b.l[i] - borrow;
            r.l[i] = (uint64_t)d;
            borrow = (uint64_t)(d >> 64) & 1;
        }
        if (borrow) {
            uint64_t carry = 0;
            for (int i = 0; i < N; i++) {
                u128 s = (u128)r.l[i] + C::MOD[i] + carry;
                r.l[i] = (uint64_t)s;
                carry = (uint64_t)(s >> 64);
            }
        }
        return r;
    }
    static T neg(const T &a) { return is_zero(a) ? a : sub(zero(), a); }
    static T dbl(const T &a) { return add(a, a); }
    // CIOS Montgomery multiplication
    static T mul(const T &a, const T &b) {
        uint64_t t[N + 2];
        memset(t, 0, sizeof t);
        for (int i = 0; i < N; i++) {
            uint64_t c = 0;
            for (int j = 0; j < N; j++) {
                u128 p = (u128)a.l[j] * b.l[i] + t[j] + c;
                t[j] = (uint64_t)p;
                c = (uint64_t)(p >> 64);
            }
            u128 s = (u128)t[N] + c;
            t[N] = (uint64_t)s;
            t[N + 1] = (uint64_t)(s >> 64);
            uint64_t m = t[0] * C::INV;
            u128 p = (u128)m * C::MOD[0] + t[0];
            c = (uint64_t)(p >> 64);
            for (int j = 1; j < N; j++) {
                p = (u128)m * C::MOD[j] + t[j] + c;
                t[j - 1] = (uint64_t)p;
                c = (uint64_t)(p >> 64);
            }
            s = (u128)t[N] + c;
            t[N - 1] = (uint64_t)s;
            t[N] = t[N + 1] + (uint64_t)(s >> 64);
        }
        T r;
        memcpy(r.l, t, sizeof r.l);
        if (t[N] || geq(r.l, C::MOD)) sub_raw(r.l, r.l, C::MOD);
        return r;
    }
    static T sqr(const T &a) { return mul(a, a); }
    static T from_raw(const uint64_t *raw) {  // canonical -> montgomery
        T a, r2;
        memcpy(a.l, raw, sizeof a.l);
        memcpy(r2.l, C::R2, sizeof r2.l);
        return mul(a, r2);
    }
    static void to_raw(const T &a, uint64_t *raw) {  // montgomery -> canonical
        T one_raw = zero();
        one_raw.l[0] = 1;
        T r = mul(a, one_raw);
        memcpy(raw, r.l, sizeof r.l);
    }
    static T pow_raw(const T &a, const uint64_t *e, int nlimbs) {
        T r = one();
        for (int i = nlimbs - 1; i >= 0; i--) {
            for (int b = 63; b >= 0; b--) {
                r = sqr(r);
                if ((e[i] >> b) & 1) r = mul(r, a);
            }
        }
        return r;
    }
    static T inv(const T &a) {  // Fermat
        uint64_t e[N];
        memcpy(e, C::MOD, sizeof e);
        // e = MOD - 2 (MOD is odd and > 2)
        uint64_t borrow = 2;
        for (int i = 0; i < N && borrow; i++) {
            uint64_t old = e[i];
            e[i] = old - borrow;
            borrow = old < borrow ? 1 : 0;
        }
        return pow_raw(a, e, N);
    }
    static bool is_canonical(const uint64_t *raw) { return !geq(raw, C::MOD); }
};

typedef F<FqTag, 6> FQ;
typedef F<FrTag, 4> FR;
typedef FQ::T fq;
typedef FR::T fr;

// ------------------------------------------------------------------------------------------
// Fq2 = Fq[u]/(u^2+1)
// ------------------------------------------------------------------------------------------
struct fq2 {
    fq c0, c1;
};

struct FQ2 {
    typedef fq2 T;
    static T zero() { return {FQ::zero(), FQ::zero()}; }
    static T one() { return {FQ::one(), FQ::zero()}; }
    static bool is_zero(const T &a) { return FQ::is_zero(a.c0) && FQ::is_zero(a.c1); }
    static bool eq(const T &a, const T &b) { return FQ::eq(a.c0, b.c0) && FQ::eq(a.c1, b.c1); }
    static T add(const T &a, const T &b) { return {FQ::add(a.c0, b.c0), FQ::add(a.c1, b.c1)}; }
    static T sub(const T &a, const T &b) { return {FQ::sub(a.c0, b.c0), FQ::sub(a.c1, b.c1)}; }
    static T neg(const T &a) { return {FQ::neg(a.c0), FQ::neg(a.c1)}; }
    static T dbl(const T &a) { return add(a, a); }
    static T mul(const T &a, const T &b) {
        fq v0 = FQ::mul(a.c0, b.c0), v1 = FQ::mul(a.c1, b.c1);
        fq t = FQ::mul(FQ::add(a.c0, a.c1), FQ::add(b.c0, b.c1));
        return {FQ::sub(v0, v1), FQ::sub(FQ::sub(t, v0), v1)};
    }
    static T sqr(const T &a) { return mul(a, a); }
    static T inv(const T &a) {
        fq n = FQ::add(FQ::sqr(a.c0), FQ::sqr(a.c1));
        fq ni = FQ::inv(n);
        return {FQ::mul(a.c0, ni), FQ::neg(FQ::mul(a.c1, ni))};
    }
    static T mul_fq(const T &a, const fq &b) { return {FQ::mul(a.c0, b), FQ::mul(a.c1, b)}; }
};

// ------------------------------------------------------------------------------------------
// Short Weierstrass y^2 = x^3 + b, Jacobian coordinates, templated over the base field.
// ------------------------------------------------------------------------------------------
template <typename FF>
struct Jac {
    typename FF::T X, Y, Z;
};
template <typename FF>
struct Aff {
    typename FF::T x, y;
    bool inf;
};

template <typename FF>
struct Curve {
    typedef typename FF::T E;
    typedef Jac<FF> J;
    typedef Aff<FF> A;
    static J identity() { return {FF::one(), FF::one(), FF::zero()}; }
    static bool is_id(const J &p) { return FF::is_zero(p.Z); }
    static J from_aff(const A &a) {
        if (a.inf) return identity();
        return {a.x, a.y, FF::one()};
    }
    static A to_aff(const J &p) {
        A r;
        if (is_id(p)) {
            r.x = FF::zero();
            r.y = FF::zero();
            r.inf = true;
            return r;
        }
        E zi = FF::inv(p.Z);
        E zi2 = FF::sqr(zi);
        r.x = FF::mul(p.X, zi2);
        r.y = FF::mul(p.Y, FF::mul(zi2, zi));
        r.inf = false;
        return r;
    }
    // dbl-2009-l (a = 0)
    static J dbl(const J &p) {
        if (is_id(p)) return p;
        E A_ = FF::sqr(p.X);
        E B = FF::sqr(p.Y);
        E C = FF::sqr(B);
        E D = FF::dbl(FF::sub(FF::sub(FF::sqr(FF::add(p.X, B)), A_), C));
        E Ee = FF::add(FF::dbl(A_), A_);
        E Fv = FF::sqr(Ee);
        J r;
        r.X = FF::sub(Fv, FF::dbl(D));
        E C8 = FF::dbl(FF::dbl(FF::dbl(C)));
        r.Y = FF::sub(FF::mul(Ee, FF::sub(D, r.X)), C8);
        r.Z = FF::dbl(FF::mul(p.Y, p.Z));
        return r;
    }
    // add-2007-bl
    static J add(const J &p, const J &q) {
        if (is_id(p)) return q;
        if (is_id(q)) return p;
        E Z1Z1 = FF::sqr(p.Z), Z2Z2 = FF::sqr(q.Z);
        E U1 = FF::mul(p.X, Z2Z2), U2 = FF::mul(q.X, Z1Z1);
        E S1 = FF::mul(FF::mul(p.Y, q.Z), Z2Z2);
        E S2 = FF::mul(FF::mul(q.Y, p.Z), Z1Z1);
        E H = FF::sub(U2, U1);
        E rr = FF::dbl(FF::sub(S2, S1));
        if (FF::is_zero(H)) {
            if (FF::is_zero(rr)) return dbl(p);
            return identity();
        }
        E I = FF::sqr(FF::dbl(H));
        E Jv = FF::mul(H, I);
        E V = FF::mul(U1, I);
        J r;
        r.X = FF::sub(FF::sub(FF::sqr(rr), Jv), FF::dbl(V));
        r.Y = FF::sub(FF::mul(rr, FF::sub(V, r.X)), FF::dbl(FF::mul(S1, Jv)));
        r.Z = FF::mul(FF::sub(FF::sub(FF::sqr(FF::add(p.Z, q.Z)), Z1Z1), Z2Z2), H);
        return r;
    }
    // madd-2007-bl (q affine, not infinity)
    static J add_mixed(const J &p, const A &q) {
        if (q.inf) return p;
        if (is_id(p)) return from_aff(q);
        E Z1Z1 = FF::sqr(p.Z);
        E U2 = FF::mul(q.x, Z1Z1);
        E S2 = FF::mul(FF::mul(q.y, p.Z), Z1Z1);
        E H = FF::sub(U2, p.X);
        E rr = FF::dbl(FF::sub(S2, p.Y));
        if (FF::is_zero(H)) {
            if (FF::is_zero(rr)) return dbl(p);
            return identity();
        }
        E HH = FF::sqr(H);
        E I = FF::dbl(FF::dbl(HH));
        E Jv = FF::mul(H, I);
        E V = FF::mul(p.X, I);
        J r;
        r.X = FF::sub(FF::sub(FF::sqr(rr), Jv), FF::dbl(V));
        r.Y = FF::sub(FF::mul(rr, FF::sub(V, r.X)), FF::dbl(FF::mul(p.Y, Jv)));
        r.Z = FF::sub(FF::sub(FF::sqr(FF::add(p.Z, H)), Z1Z1), HH);
        return r;
    }
    static J neg(const J &p) { return {p.X, FF::neg(p.Y), p.Z}; }
    static A neg(const A &p) {
        A r = p;
        if (!p.inf) r.y = FF::neg(p.y);
        return r;
    }
    static bool eq(const J &p, const J &q) {
        if (is_id(p) || is_id(q)) return is_id(p) && is_id(q);
        E Z1Z1 = FF::sqr(p.Z), Z2Z2 = FF::sqr(q.Z);
        if (!FF::eq(FF::mul(p.X, Z2Z2), FF::mul(q.X, Z1Z1))) return false;
        return FF::eq(FF::mul(FF::mul(p.Y, q.Z), Z2Z2), FF::mul(FF::mul(q.Y, p.Z), Z1Z1));
    }
    // double-and-add by a canonical scalar given as 64-bit limbs
    static J mul(const J &p, const uint64_t *k, int nlimbs) {
        J r = identity();
        for (int i = nlimbs - 1; i >= 0; i--)
            for (int b = 63; b >= 0; b--) {
                r = dbl(r);
                if ((k[i] >> b) & 1) r = add(r, p);
            }
        return r;
    }
};

typedef Curve<FQ> G1;
typedef Curve<FQ2> G2;
typedef G1::J g1j;
typedef G1::A g1a;
typedef G2::J g2j;
typedef G2::A g2a;

fq fq_b() {
    uint64_t four[6] = {4, 0, 0, 0, 0, 0};
    return FQ::from_raw(four);
}
fq2 fq2_b() {
    fq f = fq_b();
    return {f, f};
}
bool g1_on_curve(const g1a &p) {
    if (p.inf) return true;
    return FQ::eq(FQ::sqr(p.y), FQ::add(FQ::mul(FQ::sqr(p.x), p.x), fq_b()));
}
bool g2_on_curve(const g2a &p) {
    if (p.inf) return true;
    return FQ2::eq(FQ2::sqr(p.y), FQ2::add(FQ2::mul(FQ2::sqr(p.x), p.x), fq2_b()));
}

// ------------------------------------------------------------------------------------------
// Byte encodings
// ------------------------------------------------------------------------------------------
void fq_to_be(const fq &a, uint8_t *out48) {
    uint64_t raw[6];
    FQ::to_raw(a, raw);
    for (int i = 0; i < 6; i++)
        for (int b = 0; b < 8; b++) out48[47 - (i * 8 + b)] = (uint8_t)(raw[i] >> (8 * b));
}
bool fq_from_be(const uint8_t *in48, fq *out, bool mask_flags) {
    uint64_t raw[6] = {0};
    for (int i = 0; i < 48; i++) {
        uint8_t byte = in48[i];
        if (i == 0 && mask_flags) byte &= 0x1f;
        int pos = 47 - i;
        raw[pos / 8] |= (uint64_t)byte << (8 * (pos % 8));
    }
    if (!FQ::is_canonical(raw)) return false;
    *out = FQ::from_raw(raw);
    return true;
}
fr fr_from_le(const uint8_t *in32) {
    uint64_t raw[4];
    memcpy(raw, in32, 32);
    return FR::from_raw(raw);
}
void fr_raw_le(const uint8_t *in32, uint64_t raw[4]) { memcpy(raw, in32, 32); }
void fr_to_le(const fr &a, uint8_t *out32) {
    uint64_t raw[4];
    FR::to_raw(a, raw);
    memcpy(out32, raw, 32);
}

bool g1_decode(const uint8_t *in, g1a *p) {
    if (in[0] & 0x40) {
        p->inf = true;
        p->x = FQ::zero();
        p->y = FQ::zero();
        return true;
    }
    p->inf = false;
    return fq_from_be(in, &p->x, true) && fq_from_be(in + 48, &p->y, false);
}
void g1_encode(const g1a &p, uint8_t *out) {
    if (p.inf) {
        memset(out, 0, 96);
        out[0] = 0x40;
        return;
    }
    fq_to_be(p.x, out);
    fq_to_be(p.y, out + 48);
}
bool g2_decode(const uint8_t *in, g2a *p) {
    if (in[0] & 0x40) {
        p->inf = true;
        p->x = FQ2::zero();
        p->y = FQ2::zero();
        return true;
    }
    p->inf = false;
    return fq_from_be(in, &p->x.c1, true) && fq_from_be(in + 48, &p->x.c0, false) &&
           fq_from_be(in + 96, &p->y.c1, false) && fq_from_be(in + 144, &p->y.c0, false);
}
void g2_encode(const g2a &p, uint8_t *out) {
    if (p.inf) {
        memset(out, 0, 192);
        out[0] = 0x40;
        return;
    }
    fq_to_be(p.x.c1, out);
    fq_to_be(p.x.c0, out + 48);
    fq_to_be(p.y.c1, out + 96);
    fq_to_be(p.y.c0, out + 144);
}
// "lexicographically largest": y > (p-1)/2 on the canonical value
bool fq_lex_largest(const fq &y) {
    uint64_t raw[6], nraw[6];
    FQ::to_raw(y, raw);
    FQ::to_raw(FQ::neg(y), nraw);
    for (int i = 5; i >= 0; i--)
        if (raw[i] != nraw[i]) return raw[i] > nraw[i];
    return false;
}
void g1_compress(const g1a &p, uint8_t *out48) {
    if (p.inf) {
        memset(out48, 0, 48);
        out48[0] = 0xc0;
        return;
    }
    fq_to_be(p.x, out48);
    out48[0] |= 0x80;
    if (fq_lex_largest(p.y)) out48[0] |= 0x20;
}
void g2_compress(const g2a &p, uint8_t *out96) {
    if (p.inf) {
        memset(out96, 0, 96);
        out96[0] = 0xc0;
        return;
    }
    fq_to_be(p.x.c1, out96);
    fq_to_be(p.x.c0, out96 + 48);
    out96[0] |= 0x80;
    bool largest = FQ::is_zero(p.y.c1) ? fq_lex_largest(p.y.c0) : fq_lex_largest(p.y.c1);
    if (largest) out96[0] |= 0x20;
}

// Standard generators (public BLS12-381 constants)
g1a g1_gen() {
    static const uint8_t gx[48] = {0x17, 0xf1, 0xd3, 0xa7, 0x31, 0x97, 0xd7, 0x94, 0x26, 0x95, 0x63, 0x8c,
                                   0x4f, 0xa9, 0xac, 0x0f, 0xc3, 0x68, 0x8c, 0x4f, 0x97, 0x74, 0xb9, 0x05,
                                   0xa1, 0x4e, 0x3a, 0x3f, 0x17, 0x1b, 0xac, 0x58, 0x6c, 0x55, 0xe8, 0x3f,
                                   0xf9, 0x7a, 0x1a, 0xef, 0xfb, 0x3a, 0xf0, 0x0a, 0xdb, 0x22, 0xc6, 0xbb};
    static const uint8_t gy[48] = {0x08, 0xb3, 0xf4, 0x81, 0xe3, 0xaa, 0xa0, 0xf1, 0xa0, 0x9e, 0x30, 0xed,
                                   0x74, 0x1d, 0x8a, 0xe4, 0xfc, 0xf5, 0xe0, 0x95, 0xd5, 0xd0, 0x0a, 0xf6,
                                   0x00, 0xdb, 0x18, 0xcb, 0x2c, 0x04, 0xb3, 0xed, 0xd0, 0x3c, 0xc7, 0x44,
                                   0xa2, 0x88, 0x8a, 0xe4, 0x0c, 0xaa, 0x23, 0x29, 0x46, 0xc5, 0xe7, 0xe1};
    g1a g;
    g.inf = false;
    fq_from_be(gx, &g.x, false);
    fq_from_be(gy, &g.y, false);
    return g;
}
g2a g2_gen() {
    static const uint8_t x0[48] = {0x02, 0x4a, 0xa2, 0xb2, 0xf0, 0x8f, 0x0a, 0x91, 0x26, 0x08, 0x05, 0x27,
                                   0x2d, 0xc5, 0x10, 0x51, 0xc6, 0xe4, 0x7a, 0xd4, 0xfa, 0x40, 0x3b, 0x02,
                                   0xb4, 0x51, 0x0b, 0x64, 0x7a, 0xe3, 0xd1, 0x77, 0x0b, 0xac, 0x03, 0x26,
                                   0xa8, 0x05, 0xbb, 0xef, 0xd4, 0x80, 0x56, 0xc8, 0xc1, 0x21, 0xbd, 0xb8};
    static const uint8_t x1[48] = {0x13, 0xe0, 0x2b, 0x60, 0x52, 0x71, 0x9f, 0x60, 0x7d, 0xac, 0xd3, 0xa0,
                                   0x88, 0x27, 0x4f, 0x65, 0x59, 0x6b, 0xd0, 0xd0, 0x99, 0x20, 0xb6, 0x1a,
                                   0xb5, 0xda, 0x61, 0xbb, 0xdc, 0x7f, 0x50, 0x49, 0x33, 0x4c, 0xf1, 0x12,
                                   0x13, 0x94, 0x5d, 0x57, 0xe5, 0xac, 0x7d, 0x05, 0x5d, 0x04, 0x2b, 0x7e};
    static const uint8_t y0[48] = {0x0c, 0xe5, 0xd5, 0x27, 0x72, 0x7d, 0x6e, 0x11, 0x8c, 0xc9, 0xcd, 0xc6,
                                   0xda, 0x2e, 0x35, 0x1a, 0xad, 0xfd, 0x9b, 0xaa, 0x8c, 0xbd, 0xd3, 0xa7,
                                   0x6d, 0x42, 0x9a, 0x69, 0x51, 0x60, 0xd1, 0x2c, 0x92, 0x3a, 0xc9, 0xcc,
                                   0x3b, 0xac, 0xa2, 0x89, 0xe1, 0x93, 0x54, 0x86, 0x08, 0xb8, 0x28, 0x01};
    static const uint8_t y1[48] = {0x06, 0x06, 0xc4, 0xa0, 0x2e, 0xa7, 0x34, 0xcc, 0x32, 0xac, 0xd2, 0xb0,
                                   0x2b, 0xc2, 0x8b, 0x99, 0xcb, 0x3e, 0x28, 0x7e, 0x85, 0xa7, 0x63, 0xaf,
                                   0x26, 0x74, 0x92, 0xab, 0x57, 0x2e, 0x99, 0xab, 0x3f, 0x37, 0x0d, 0x27,
                                   0x5c, 0xec, 0x1d, 0xa1, 0xaa, 0xa9, 0x07, 0x5f, 0xf0, 0x5f, 0x79, 0xbe};
    g2a g;
    g.inf = false;
    fq_from_be(x0, &g.x.c0, false);
    fq_from_be(x1, &g.x.c1, false);
    fq_from_be(y0, &g.y.c0, false);
    fq_from_be(y1, &g.y.c1, false);
    return g;
}

// ------------------------------------------------------------------------------------------
// Fr helpers: roots of unity (bellman: GENERATOR = 7, S = 32, ROOT_OF_UNITY = 7^((r-1)/2^32))
// ------------------------------------------------------------------------------------------
fr fr_from_u64(uint64_t v) {
    uint64_t raw[4] = {v, 0, 0, 0};
    return FR::from_raw(raw);
}
fr fr_root_of_unity_2_32() {
    // t = (r - 1) >> 32
    uint64_t t[4];
    const uint64_t *m = Consts<FrTag, 4>::MOD;
    uint64_t rm1[4] = {m[0] - 1, m[1], m[2], m[3]};
    for (int i = 0; i < 4; i++) t[i] = (rm1[i] >> 32) | (i < 3 ? (rm1[i + 1] << 32) : 0);
    return FR::pow_raw(fr_from_u64(7), t, 4);
}
fr fr_omega(unsigned log_n) {
    fr w = fr_root_of_unity_2_32();
    for (unsigned i = log_n; i < 32; i++) w = FR::sqr(w);
    return w;
}
fr fr_pow_u64(const fr &a, uint64_t e) { return FR::pow_raw(a, &e, 1); }

int g_threads = 0;
int nthreads() { return g_threads > 0 ? g_threads : omp_get_max_threads(); }

// ------------------------------------------------------------------------------------------
// Evaluation domain (bellman EvaluationDomain::{fft, ifft, coset_fft, icoset_fft})
// ------------------------------------------------------------------------------------------
uint64_t bitrev(uint64_t x, unsigned bits) {
    uint64_t r = 0;
    for (unsigned i = 0; i < bits; i++) r |= ((x >> i) & 1) << (bits - 1 - i);
    return r;
}
// serial_fft with bit reversal first then DIT stages; stages parallelised with OpenMP.
void fft_inplace(std::vector<fr> &a, const fr &omega, unsigned log_n) {
    uint64_t n = 1ULL << log_n;
    for (uint64_t k = 0; k < n; k++) {
        uint64_t rk = bitrev(k, log_n);
        if (k < rk) std::swap(a[k], a[rk]);
    }
    // twiddle table omega^i, i < n/2
    std::vector<fr> tw(n / 2 > 0 ? n / 2 : 1);
    tw[0] = FR::one();
    for (uint64_t i = 1; i < n / 2; i++) tw[i] = FR::mul(tw[i - 1], omega);
    int nt = nthreads();
    for (uint64_t m = 1; m < n; m *= 2) {
        uint64_t stride = n / (2 * m);
#pragma omp parallel for num_threads(nt) schedule(static) if (n >= 4096)
        for (int64_t idx = 0; idx < (int64_t)(n / 2); idx++) {
            uint64_t k = (idx / m) * 2 * m;
            uint64_t j = idx % m;
            fr t = FR::mul(a[k + j + m], tw[j * stride]);
            fr u = a[k + j];
            a[k + j + m] = FR::sub(u, t);
            a[k + j] = FR::add(u, t);
        }
    }
}
void domain_op(std::vector<fr> &a, unsigned log_n, int kind) {
    uint64_t n = 1ULL << log_n;
    fr omega = fr_omega(log_n);
    fr g = fr_from_u64(7);
    int nt = nthreads();
    if (kind == 0) {
        fft_inplace(a, omega, log_n);
    } else if (kind == 1 || kind == 3) {
        fft_inplace(a, FR::inv(omega), log_n);
        fr minv = FR::inv(fr_from_u64(n));
        if (kind == 1) {
#pragma omp parallel for num_threads(nt)
            for (int64_t i = 0; i < (int64_t)n; i++) a[i] = FR::mul(a[i], minv);
        } else {
            // icoset: ifft then distribute powers of g^-1 (bellman: distribute_powers(geninv))
            fr gi = FR::inv(g);
#pragma omp parallel num_threads(nt)
            {
                int t = omp_get_thread_num(), T = omp_get_num_threads();
                uint64_t chunk = (n + T - 1) / T, lo = t * chunk, hi = lo + chunk < n ? lo + chunk : n;
                if (lo < hi) {
                    fr w = FR::mul(fr_pow_u64(gi, lo), minv);
                    for (uint64_t i = lo; i < hi; i++) {
                        a[i] = FR::mul(a[i], w);
                        w = FR::mul(w, gi);
                    }
                }
            }
        }
    } else if (kind == 2) {
#pragma omp parallel num_threads(nt)
        {
            int t = omp_get_thread_num(), T = omp_get_num_threads();
            uint64_t chunk = (n + T - 1) / T, lo = t * chunk, hi = lo + chunk < n ? lo + chunk : n;
            if (lo < hi) {
                fr w = fr_pow_u64(g, lo);
                for (uint64_t i = lo; i < hi; i++) {
                    a[i] = FR::mul(a[i], w);
                    w = FR::mul(w, g);
                }
            }
        }
        fft_inplace(a, omega, log_n);
    }
}

// ------------------------------------------------------------------------------------------
// Multiexp: bellman-style unsigned-window Pippenger per thread chunk, chunks summed.
// ------------------------------------------------------------------------------------------
template <typename CV>
typename CV::J pippenger_serial(const typename CV::A *bases, const uint64_t (*k)[4], size_t n) {
    typedef typename CV::J J;
    if (n == 0) return CV::identity();
    unsigned c = n < 32 ? 3 : 0;
    if (!c) {
        double l = 0;
        size_t x = n;
        // c = ceil(ln n) (bellman multiexp heuristic)
        l = __builtin_log((double)x);
        c = (unsigned)__builtin_ceil(l);
    }
    J acc = CV::identity();
    std::vector<J> buckets((1u << c) - 1);
    unsigned nwin = (256 + c - 1) / c;
    for (int w = (int)nwin - 1; w >= 0; w--) {
        for (unsigned i = 0; i < c; i++) acc = CV::dbl(acc);
        for (auto &b : buckets) b = CV::identity();
        unsigned bit0 = w * c;
        for (size_t i = 0; i < n; i++) {
            // extract c bits starting at bit0
            uint64_t d = 0;
            for (unsigned b = 0; b < c; b++) {
                unsigned pos = bit0 + b;
                if (pos >= 256) break;
                d |= ((k[i][pos / 64] >> (pos % 64)) & 1ULL) << b;
            }
            if (d) buckets[d - 1] = CV::add_mixed(buckets[d - 1], bases[i]);
        }
        J run = CV::identity(), sum = CV::identity();
        for (int b = (int)buckets.size() - 1; b >= 0; b--) {
            run = CV::add(run, buckets[b]);
            sum = CV::add(sum, run);
        }
        acc = CV::add(acc, sum);
    }
    return acc;
}
template <typename CV>
typename CV::J pippenger(const typename CV::A *bases, const uint64_t (*k)[4], size_t n) {
    int nt = nthreads();
    if (n < 1024 || nt == 1) return pippenger_serial<CV>(bases, k, n);
    std::vector<typename CV::J> part(nt);
    size_t chunk = (n + nt - 1) / nt;
#pragma omp parallel for num_threads(nt) schedule(static, 1)
    for (int t = 0; t < nt; t++) {
        size_t lo = t * chunk, hi = lo + chunk < n ? lo + chunk : n;
        part[t] = lo < hi ? pippenger_serial<CV>(bases + lo, k + lo, hi - lo) : CV::identity();
    }
    typename CV::J r = CV::identity();
    for (int t = 0; t < nt; t++) r = CV::add(r, part[t]);
    return r;
}

// ------------------------------------------------------------------------------------------
// Fq12 = Fq[w]/(w^12 - 2 w^6 + 2) (the "twist into E(Fq12)" representation); pairing.
// Fq2 embeds via u -> w^6 - 1.  G2 point (x, y) maps to (x / w^2, y / w^3) on y^2 = x^3 + 4.
// ------------------------------------------------------------------------------------------
struct fq12 {
    fq c[12];
};
fq12 f12_zero() {
    fq12 r;
    for (int i = 0; i < 12; i++) r.c[i] = FQ::zero();
    return r;
}
fq12 f12_one() {
    fq12 r = f12_zero();
    r.c[0] = FQ::one();
    return r;
}
fq12 f12_add(const fq12 &a, const fq12 &b) {
    fq12 r;
    for (int i = 0; i < 12; i++) r.c[i] = FQ::add(a.c[i], b.c[i]);
    return r;
}
fq12 f12_sub(const fq12 &a, const fq12 &b) {
    fq12 r;
    for (int i = 0; i < 12; i++) r.c[i] = FQ::sub(a.c[i], b.c[i]);
    return r;
}
fq12 f12_mul(const fq12 &a, const fq12 &b) {
    fq t[23];
    for (int i = 0; i < 23; i++) t[i] = FQ::zero();
    for (int i = 0; i < 12; i++) {
        if (FQ::is_zero(a.c[i])) continue;
        for (int j = 0; j < 12; j++) t[i + j] = FQ::add(t[i + j], FQ::mul(a.c[i], b.c[j]));
    }
    for (int k = 22; k >= 12; k--) {  // w^k = w^(k-12) * (2 w^6 - 2)
        fq two = FQ::dbl(t[k]);
        t[k - 6] = FQ::add(t[k - 6], two);
        t[k - 12] = FQ::sub(t[k - 12], two);
    }
    fq12 r;
    for (int i = 0; i < 12; i++) r.c[i] = t[i];
    return r;
}
bool f12_eq(const fq12 &a, const fq12 &b) {
    for (int i = 0; i < 12; i++)
        if (!FQ::eq(a.c[i], b.c[i])) return false;
    return true;
}
fq12 f12_embed_fq2(const fq2 &a) {  // a0 + a1 u -> (a0 - a1) + a1 w^6
    fq12 r = f12_zero();
    r.c[0] = FQ::sub(a.c0, a.c1);
    r.c[6] = a.c1;
    return r;
}
fq12 f12_from_fq(const fq &a) {
    fq12 r = f12_zero();
    r.c[0] = a;
    return r;
}
// w^-1 = (w^11 - 2 w^5) / (-2)   since w^12 - 2 w^6 = -2  =>  w (w^11 - 2 w^5) = -2
fq12 f12_winv() {
    fq12 r = f12_zero();
    fq m2inv = FQ::inv(FQ::neg(FQ::dbl(FQ::one())));
    r.c[11] = m2inv;
    r.c[5] = FQ::neg(FQ::dbl(m2inv));
    return r;
}
fq12 f12_pow_big(const fq12 &a, const std::vector<uint64_t> &e) {
    fq12 r = f12_one();
    for (int i = (int)e.size() - 1; i >= 0; i--)
        for (int b = 63; b >= 0; b--) {
            r = f12_mul(r, r);
            if ((e[i] >> b) & 1) r = f12_mul(r, a);
        }
    return r;
}
// big integer helpers for the final exponent (p^12 - 1) / r
std::vector<uint64_t> big_mul(const std::vector<uint64_t> &a, const std::vector<uint64_t> &b) {
    std::vector<uint64_t> r(a.size() + b.size(), 0);
    for (size_t i = 0; i < a.size(); i++) {
        uint64_t c = 0;
        for (size_t j = 0; j < b.size(); j++) {
            u128 p = (u128)a[i] * b[j] + r[i + j] + c;
            r[i + j] = (uint64_t)p;
            c = (uint64_t)(p >> 64);
        }
        r[i + b.size()] = c;
    }
    while (r.size() > 1 && r.back() == 0) r.pop_back();
    return r;
}
// divide by a 4-limb divisor using simple long division on bits (slow but only once)
std::vector<uint64_t> big_div(std::vector<uint64_t> num, const std::vector<uint64_t> &den) {
    size_t nb = num.size() * 64;
    std::vector<uint64_t> q(num.size(), 0), rem(den.size() + 1, 0);
    for (int64_t bit = (int64_t)nb - 1; bit >= 0; bit--) {
        // rem = rem*2 + bit
        uint64_t carry = (num[bit / 64] >> (bit % 64)) & 1;
        for (size_t i = 0; i < rem.size(); i++) {
            uint64_t nc = rem[i] >> 63;
            rem[i] = (rem[i] << 1) | carry;
            carry = nc;
        }
        // if rem >= den: rem -= den
        bool ge = true;
        for (int64_t i = (int64_t)rem.size() - 1; i >= 0; i--) {
            uint64_t dv = (size_t)i < den.size() ? den[i] : 0;
            if (rem[i] != dv) {
                ge = rem[i] > dv;
                break;
            }
        }
        if (ge) {
            uint64_t borrow = 0;
            for (size_t i = 0; i < rem.size(); i++) {
                uint64_t dv = i < den.size() ? den[i] : 0;
                u128 d = (u128)rem[i] - dv - borrow;
                rem[i] = (uint64_t)d;
                borrow = (uint64_t)(d >> 64) & 1;
            }
            q[bit / 64] |= 1ULL << (bit % 64);
        }
    }
    while (q.size() > 1 && q.back() == 0) q.pop_back();
    return q;
}
const std::vector<uint64_t> &final_exponent() {
    static std::vector<uint64_t> e;
    static bool init = false;
#pragma omp critical(or_final_exp)
    if (!init) {
        std::vector<uint64_t> p(Consts<FqTag, 6>::MOD, Consts<FqTag, 6>::MOD + 6);
        std::vector<uint64_t> p12 = {1};
        for (int i = 0; i < 12; i++) p12 = big_mul(p12, p);
        // p^12 - 1
        for (size_t i = 0; i < p12.size(); i++) {
            if (p12[i]-- != 0) break;
        }
        std::vector<uint64_t> r(Consts<FrTag, 4>::MOD, Consts<FrTag, 4>::MOD + 4);
        e = big_div(p12, r);
        init = true;
    }
    return e;
}
// Miller loop over |x| = 0xd201000000010000 (py_ecc-style; sign ignored -> a fixed power of
// the optimal ate pairing, still bilinear and non-degenerate, which is all a product check needs)
fq12 miller_loop(const g2a &Q, const g1a &P) {
    if (Q.inf || P.inf) return f12_one();
    static const uint64_t ATE = 0xd201000000010000ULL;
    fq12 winv = f12_winv();
    fq12 winv2 = f12_mul(winv, winv), winv3 = f12_mul(winv2, winv);
    fq12 xP = f12_from_fq(P.x), yP = f12_from_fq(P.y);
    auto line = [&](const g2a &R, const fq2 &slope) {
        // l(P) = m12 (xP - xR12) - (yP - yR12)
        fq12 m12 = f12_mul(f12_embed_fq2(slope), winv);
        fq12 xR = f12_mul(f12_embed_fq2(R.x), winv2);
        fq12 yR = f12_mul(f12_embed_fq2(R.y), winv3);
        return f12_sub(f12_mul(m12, f12_sub(xP, xR)), f12_sub(yP, yR));
    };
    g2a R = Q;
    fq12 f = f12_one();
    for (int i = 62; i >= 0; i--) {
        // doubling: slope = 3x^2 / 2y
        fq2 x2 = FQ2::sqr(R.x);
        fq2 slope = FQ2::mul(FQ2::add(FQ2::dbl(x2), x2), FQ2::inv(FQ2::dbl(R.y)));
        f = f12_mul(f12_mul(f, f), line(R, slope));
        fq2 nx = FQ2::sub(FQ2::sqr(slope), FQ2::dbl(R.x));
        fq2 ny = FQ2::sub(FQ2::mul(slope, FQ2::sub(R.x, nx)), R.y);
        R.x = nx;
        R.y = ny;
        if ((ATE >> i) & 1) {
            fq2 s2 = FQ2::mul(FQ2::sub(Q.y, R.y), FQ2::inv(FQ2::sub(Q.x, R.x)));
            f = f12_mul(f, line(R, s2));
            fq2 ax = FQ2::sub(FQ2::sub(FQ2::sqr(s2), R.x), Q.x);
            fq2 ay = FQ2::sub(FQ2::mul(s2, FQ2::sub(R.x, ax)), R.y);
            R.x = ax;
            R.y = ay;
        }
    }
    return f;
}

}  // namespace

// ==========================================================================================
// Groth16 parameters (bellman generator) -- opaque struct
// ==========================================================================================
struct or_params {
    uint64_t n, n_in, n_aux, d;
    unsigned log_d;
    fr tau, alpha, beta, gamma, delta;
    std::vector<fr> at, bt, ct;  // per variable QAP evaluations at tau
    std::vector<uint8_t> a_aux_density, b_in_density, b_aux_density;
    std::vector<g1a> h, l, a, b_g1, ic;
    std::vector<g2a> b_g2;
    g1a alpha_g1, beta_g1, delta_g1;
    g2a beta_g2, gamma_g2, delta_g2;
};

namespace {
std::vector<g1a> g1_fixed_base_vec(const std::vector<fr> &k) {
    std::vector<g1a> out(k.size());
    g1j g = G1::from_aff(g1_gen());
    int nt = nthreads();
#pragma omp parallel for num_threads(nt) schedule(dynamic, 64)
    for (int64_t i = 0; i < (int64_t)k.size(); i++) {
        uint64_t raw[4];
        FR::to_raw(k[i], raw);
        out[i] = G1::to_aff(G1::mul(g, raw, 4));
    }
    return out;
}
std::vector<g2a> g2_fixed_base_vec(const std::vector<fr> &k) {
    std::vector<g2a> out(k.size());
    g2j g = G2::from_aff(g2_gen());
    int nt = nthreads();
#pragma omp parallel for num_threads(nt) schedule(dynamic, 16)
    for (int64_t i = 0; i < (int64_t)k.size(); i++) {
        uint64_t raw[4];
        FR::to_raw(k[i], raw);
        out[i] = G2::to_aff(G2::mul(g, raw, 4));
    }
    return out;
}
fr lc_eval(const or_r1cs *cs, int m, uint64_t row, const std::vector<fr> &z) {
    fr acc = FR::zero();
    for (uint64_t e = cs->row_ptr[m][row]; e < cs->row_ptr[m][row + 1]; e++) {
        fr c = fr_from_le(cs->coeff[m] + 32 * e);
        acc = FR::add(acc, FR::mul(c, z[cs->col[m][e]]));
    }
    return acc;
}
std::vector<fr> load_z(const or_r1cs *cs, const uint8_t *z32) {
    uint64_t nv = cs->num_inputs + cs->num_aux;
    std::vector<fr> z(nv);
    for (uint64_t i = 0; i < nv; i++) z[i] = fr_from_le(z32 + 32 * i);
    return z;
}
unsigned domain_log(uint64_t rows) {
    unsigned lg = 0;
    while ((1ULL << lg) < rows) lg++;
    return lg;
}
}  // namespace

extern "C" {

/* Poseidon, literal form (oracle/poseidon_ref.py restated with 64-bit-limb Montgomery Fr and OpenMP, for
 * the tree builders' CPU baseline and large checks).  PARITY UNPINNED.  rc: (rf + rp) * t canonical
 * constants, mds: t * t (state' = state * M), tag = 2^arity - 1, digest = state[1];
 * out[i] = hash(in[i * arity .. i * arity + arity - 1]).  Returns -1 on a non-canonical input. */
int or_poseidon_hash(unsigned arity, const uint8_t *rc32, const uint8_t *mds32, unsigned rf, unsigned rp,
                     const uint8_t *in32, uint64_t n, uint8_t *out32) {
    const unsigned t = arity + 1;
    if (t > 17) return -1;
    std::vector<fr> rc((size_t)(rf + rp) * t), m((size_t)t * t);
    for (size_t i = 0; i < rc.size(); i++) rc[i] = fr_from_le(rc32 + 32 * i);
    for (size_t i = 0; i < m.size(); i++) m[i] = fr_from_le(mds32 + 32 * i);
    uint8_t tagb[32] = {0};
    const uint64_t tag = (1ull << arity) - 1;
    memcpy(tagb, &tag, 8);
    const fr ftag = fr_from_le(tagb);
    int bad = 0;
    const int nt = nthreads();
#pragma omp parallel for num_threads(nt) schedule(static) reduction(| : bad) if (n >= 64)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        fr s[17], nx[17];
        s[0] = ftag;
        for (unsigned j = 0; j < arity; j++) {
            uint64_t raw[4];
            memcpy(raw, in32 + 32 * ((uint64_t)i * arity + j), 32);
            if (!FR::is_canonical(raw)) bad |= 1;
            s[j + 1] = FR::from_raw(raw);
        }
        unsigned k = 0;
        for (unsigned r = 0; r < rf + rp; r++) {
            const bool full = r < rf / 2 || r >= rf / 2 + rp;
            for (unsigned j = 0; j < t; j++) s[j] = FR::add(s[j], rc[k + j]);
            k += t;
            for (unsigned j = 0; j < (full ? t : 1u); j++) {
                fr x2 = FR::mul(s[j], s[j]);
                s[j] = FR::mul(FR::mul(x2, x2), s[j]);
            }
            for (unsigned j = 0; j < t; j++) {
                fr acc = FR::zero();
                for (unsigned q = 0; q < t; q++) acc = FR::add(acc, FR::mul(s[q], m[(size_t)q * t + j]));
                nx[j] = acc;
            }
            for (unsigned j = 0; j < t; j++) s[j] = nx[j];
        }
        fr_to_le(s[1], out32 + 32 * (uint64_t)i);
    }
    return bad ? -1 : 0;
}

/* The same hash in the optimised (sparse) form -- constants from poseidon_ref.sparse_form, derived there
 * independently of the GPU library -- for a CPU baseline with the operation count Filecoin's CPU
 * implementation has: folded partial-round constants, 2t - 1 products per partial round.
 * first / last: (rf / 2) * t, part: rp, mds / dense: t * t, rows: (rp - 1) * (t + t - 1). */
int or_poseidon_hash_sparse(unsigned arity, unsigned rf, unsigned rp, const uint8_t *first32, const uint8_t *part32,
                            const uint8_t *last32, const uint8_t *mds32, const uint8_t *rows32, const uint8_t *dense32,
                            const uint8_t *in32, uint64_t n, uint8_t *out32) {
    const unsigned t = arity + 1, half = rf / 2;
    if (t > 17) return -1;
    auto vec = [](const uint8_t *b, size_t cnt) {
        std::vector<fr> v(cnt);
        for (size_t i = 0; i < cnt; i++) v[i] = fr_from_le(b + 32 * i);
        return v;
    };
    const std::vector<fr> cf = vec(first32, (size_t)half * t), cp = vec(part32, rp), cl = vec(last32, (size_t)half * t),
                          m = vec(mds32, (size_t)t * t), rows = vec(rows32, (size_t)(rp - 1) * (2 * t - 1)),
                          dn = vec(dense32, (size_t)t * t);
    uint8_t tagb[32] = {0};
    const uint64_t tag = (1ull << arity) - 1;
    memcpy(tagb, &tag, 8);
    const fr ftag = fr_from_le(tagb);
    int bad = 0;
    const int nt = nthreads();
#pragma omp parallel for num_threads(nt) schedule(static) reduction(| : bad) if (n >= 64)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        fr s[17], nx[17];
        s[0] = ftag;
        for (unsigned j = 0; j < arity; j++) {
            uint64_t raw[4];
            memcpy(raw, in32 + 32 * ((uint64_t)i * arity + j), 32);
            if (!FR::is_canonical(raw)) bad |= 1;
            s[j + 1] = FR::from_raw(raw);
        }
        auto sbox = [](const fr &x) {
            fr x2 = FR::mul(x, x);
            return FR::mul(FR::mul(x2, x2), x);
        };
        auto matv = [&](const std::vector<fr> &a) {
            for (unsigned r = 0; r < t; r++) {
                fr acc = FR::zero();
                for (unsigned q = 0; q < t; q++) acc = FR::add(acc, FR::mul(a[(size_t)r * t + q], s[q]));
                nx[r] = acc;
            }
            for (unsigned r = 0; r < t; r++) s[r] = nx[r];
        };
        for (unsigned r = 0; r < half; r++) {
            for (unsigned j = 0; j < t; j++) s[j] = sbox(FR::add(s[j], cf[(size_t)r * t + j]));
            matv(m);
        }
        for (unsigned k = 0; k + 1 < rp; k++) {
            const fr *row = &rows[(size_t)k * (2 * t - 1)];
            s[0] = sbox(FR::add(s[0], cp[k]));
            fr n0 = FR::zero();
            for (unsigned q = 0; q < t; q++) n0 = FR::add(n0, FR::mul(row[q], s[q]));
            for (unsigned j = 1; j < t; j++) s[j] = FR::add(s[j], FR::mul(row[t + j - 1], s[0]));
            s[0] = n0;
        }
        s[0] = sbox(FR::add(s[0], cp[rp - 1]));
        matv(dn);
        for (unsigned r = 0; r < half; r++) {
            for (unsigned j = 0; j < t; j++) s[j] = sbox(FR::add(s[j], cl[(size_t)r * t + j]));
            matv(m);
        }
        fr_to_le(s[1], out32 + 32 * (uint64_t)i);
    }
    return bad ? -1 : 0;
}

void or_set_threads(int n) { g_threads = n; }
int or_get_threads(void) { return nthreads(); }

void or_fr_mul(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
    fr_to_le(FR::mul(fr_from_le(a), fr_from_le(b)), out);
}
void or_fr_inv(const uint8_t a[32], uint8_t out[32]) { fr_to_le(FR::inv(fr_from_le(a)), out); }
void or_fr_root_of_unity(unsigned log_n, uint8_t out[32]) { fr_to_le(fr_omega(log_n), out); }
void or_g1_generator(uint8_t out96[96]) { g1_encode(g1_gen(), out96); }
void or_g2_generator(uint8_t out192[192]) { g2_encode(g2_gen(), out192); }

int or_g1_mul(const uint8_t p96[96], const uint8_t s[32], uint8_t out96[96]) {
    g1a p;
    if (!g1_decode(p96, &p)) return -1;
    uint64_t k[4];
    fr_raw_le(s, k);
    g1_encode(G1::to_aff(G1::mul(G1::from_aff(p), k, 4)), out96);
    return 0;
}
int or_g2_mul(const uint8_t p192[192], const uint8_t s[32], uint8_t out192[192]) {
    g2a p;
    if (!g2_decode(p192, &p)) return -1;
    uint64_t k[4];
    fr_raw_le(s, k);
    g2_encode(G2::to_aff(G2::mul(G2::from_aff(p), k, 4)), out192);
    return 0;
}
int or_g1_add(const uint8_t a96[96], const uint8_t b96[96], uint8_t out96[96]) {
    g1a a, b;
    if (!g1_decode(a96, &a) || !g1_decode(b96, &b)) return -1;
    g1_encode(G1::to_aff(G1::add(G1::from_aff(a), G1::from_aff(b))), out96);
    return 0;
}
int or_g2_add(const uint8_t a192[192], const uint8_t b192[192], uint8_t out192[192]) {
    g2a a, b;
    if (!g2_decode(a192, &a) || !g2_decode(b192, &b)) return -1;
    g2_encode(G2::to_aff(G2::add(G2::from_aff(a), G2::from_aff(b))), out192);
    return 0;
}
int or_g1_compress(const uint8_t p96[96], uint8_t out48[48]) {
    g1a p;
    if (!g1_decode(p96, &p)) return -1;
    g1_compress(p, out48);
    return 0;
}
int or_g2_compress(const uint8_t p192[192], uint8_t out96[96]) {
    g2a p;
    if (!g2_decode(p192, &p)) return -1;
    g2_compress(p, out96);
    return 0;
}
int or_g1_on_curve(const uint8_t p96[96]) {
    g1a p;
    return g1_decode(p96, &p) && g1_on_curve(p);
}
int or_g2_on_curve(const uint8_t p192[192]) {
    g2a p;
    return g2_decode(p192, &p) && g2_on_curve(p);
}
void or_g1_fixed_base(const uint8_t *k32, size_t n, uint8_t *out96) {
    std::vector<fr> k(n);
    for (size_t i = 0; i < n; i++) k[i] = fr_from_le(k32 + 32 * i);
    std::vector<g1a> pts = g1_fixed_base_vec(k);
    for (size_t i = 0; i < n; i++) g1_encode(pts[i], out96 + 96 * i);
}
void or_g2_fixed_base(const uint8_t *k32, size_t n, uint8_t *out192) {
    std::vector<fr> k(n);
    for (size_t i = 0; i < n; i++) k[i] = fr_from_le(k32 + 32 * i);
    std::vector<g2a> pts = g2_fixed_base_vec(k);
    for (size_t i = 0; i < n; i++) g2_encode(pts[i], out192 + 192 * i);
}

void or_ntt(uint8_t *data32, unsigned log_n, int kind) {
    uint64_t n = 1ULL << log_n;
    std::vector<fr> a(n);
    for (uint64_t i = 0; i < n; i++) a[i] = fr_from_le(data32 + 32 * i);
    domain_op(a, log_n, kind);
    for (uint64_t i = 0; i < n; i++) fr_to_le(a[i], data32 + 32 * i);
}

int or_msm_g1(const uint8_t *bases96, const uint8_t *scalars32, size_t n, uint8_t out96[96]) {
    std::vector<g1a> b(n);
    std::vector<uint64_t> k(4 * n);
    for (size_t i = 0; i < n; i++) {
        if (!g1_decode(bases96 + 96 * i, &b[i])) return -1;
        memcpy(&k[4 * i], scalars32 + 32 * i, 32);
    }
    g1_encode(G1::to_aff(pippenger<G1>(b.data(), (const uint64_t(*)[4])k.data(), n)), out96);
    return 0;
}
int or_msm_g2(const uint8_t *bases192, const uint8_t *scalars32, size_t n, uint8_t out192[192]) {
    std::vector<g2a> b(n);
    std::vector<uint64_t> k(4 * n);
    for (size_t i = 0; i < n; i++) {
        if (!g2_decode(bases192 + 192 * i, &b[i])) return -1;
        memcpy(&k[4 * i], scalars32 + 32 * i, 32);
    }
    g2_encode(G2::to_aff(pippenger<G2>(b.data(), (const uint64_t(*)[4])k.data(), n)), out192);
    return 0;
}
int or_msm_g1_naive(const uint8_t *bases96, const uint8_t *scalars32, size_t n, uint8_t out96[96]) {
    g1j acc = G1::identity();
    for (size_t i = 0; i < n; i++) {
        g1a b;
        if (!g1_decode(bases96 + 96 * i, &b)) return -1;
        uint64_t k[4];
        memcpy(k, scalars32 + 32 * i, 32);
        acc = G1::add(acc, G1::mul(G1::from_aff(b), k, 4));
    }
    g1_encode(G1::to_aff(acc), out96);
    return 0;
}

int or_r1cs_satisfied(const or_r1cs *cs, const uint8_t *z32) {
    std::vector<fr> z = load_z(cs, z32);
    for (uint64_t j = 0; j < cs->num_constraints; j++) {
        fr a = lc_eval(cs, 0, j, z), b = lc_eval(cs, 1, j, z), c = lc_eval(cs, 2, j, z);
        if (!FR::eq(FR::mul(a, b), c)) return 0;
    }
    return 1;
}

// bellman groth16::generate_parameters with g1 = G1 generator, g2 = G2 generator
or_params *or_groth16_keygen(const or_r1cs *cs, const uint8_t toxic[5 * 32]) {
    or_params *P = new or_params();
    P->n = cs->num_constraints;
    P->n_in = cs->num_inputs;
    P->n_aux = cs->num_aux;
    P->log_d = domain_log(P->n + P->n_in);
    P->d = 1ULL << P->log_d;
    P->tau = fr_from_le(toxic);
    P->alpha = fr_from_le(toxic + 32);
    P->beta = fr_from_le(toxic + 64);
    P->gamma = fr_from_le(toxic + 96);
    P->delta = fr_from_le(toxic + 128);
    uint64_t d = P->d, nv = P->n_in + P->n_aux;
    // powers of tau -> Lagrange coefficients via ifft
    std::vector<fr> lag(d);
    lag[0] = FR::one();
    for (uint64_t i = 1; i < d; i++) lag[i] = FR::mul(lag[i - 1], P->tau);
    fr tau_d = FR::mul(lag[d - 1], P->tau);
    fr t_tau = FR::sub(tau_d, FR::one());
    fr delta_inv = FR::inv(P->delta), gamma_inv = FR::inv(P->gamma);
    // h query: tau^i * t(tau) / delta, i < d - 1
    std::vector<fr> hk(d - 1);
    fr coeff = FR::mul(t_tau, delta_inv);
    for (uint64_t i = 0; i + 1 < d; i++) hk[i] = FR::mul(lag[i], coeff);
    domain_op(lag, P->log_d, 1);
    // QAP evaluations per variable
    P->at.assign(nv, FR::zero());
    P->bt.assign(nv, FR::zero());
    P->ct.assign(nv, FR::zero());
    P->a_aux_density.assign(P->n_aux, 0);
    P->b_in_density.assign(P->n_in, 0);
    P->b_aux_density.assign(P->n_aux, 0);
    std::vector<fr> *acc[3] = {&P->at, &P->bt, &P->ct};
    for (int m = 0; m < 3; m++)
        for (uint64_t j = 0; j < P->n; j++)
            for (uint64_t e = cs->row_ptr[m][j]; e < cs->row_ptr[m][j + 1]; e++) {
                uint32_t v = cs->col[m][e];
                fr c = fr_from_le(cs->coeff[m] + 32 * e);
                (*acc[m])[v] = FR::add((*acc[m])[v], FR::mul(c, lag[j]));
                if (m == 0 && v >= P->n_in) P->a_aux_density[v - P->n_in] = 1;
                if (m == 1) {
                    if (v < P->n_in)
                        P->b_in_density[v] = 1;
                    else
                        P->b_aux_density[v - P->n_in] = 1;
                }
            }
    // input constraints x_i * 0 = 0 appended after the circuit's constraints
    for (uint64_t i = 0; i < P->n_in; i++) P->at[i] = FR::add(P->at[i], lag[P->n + i]);
    // scalars for each query
    std::vector<fr> ka, kb, kl, kic;
    for (uint64_t v = 0; v < nv; v++) {
        if (!FR::is_zero(P->at[v])) ka.push_back(P->at[v]);
        if (!FR::is_zero(P->bt[v])) kb.push_back(P->bt[v]);
        fr ext = FR::add(FR::add(FR::mul(P->beta, P->at[v]), FR::mul(P->alpha, P->bt[v])), P->ct[v]);
        if (v < P->n_in)
            kic.push_back(FR::mul(ext, gamma_inv));
        else
            kl.push_back(FR::mul(ext, delta_inv));
    }
    P->h = g1_fixed_base_vec(hk);
    P->l = g1_fixed_base_vec(kl);
    P->a = g1_fixed_base_vec(ka);
    P->b_g1 = g1_fixed_base_vec(kb);
    P->b_g2 = g2_fixed_base_vec(kb);
    P->ic = g1_fixed_base_vec(kic);
    std::vector<fr> vk1 = {P->alpha, P->beta, P->delta};
    std::vector<g1a> v1 = g1_fixed_base_vec(vk1);
    P->alpha_g1 = v1[0];
    P->beta_g1 = v1[1];
    P->delta_g1 = v1[2];
    std::vector<fr> vk2 = {P->beta, P->gamma, P->delta};
    std::vector<g2a> v2 = g2_fixed_base_vec(vk2);
    P->beta_g2 = v2[0];
    P->gamma_g2 = v2[1];
    P->delta_g2 = v2[2];
    return P;
}
// Load a proving key produced elsewhere (bellman layout, wire encodings).  Densities come from the
// R1CS (a variable is dense when it appears in the matrix), as in bellman's prover.  The trapdoor
// fields stay empty: or_groth16_trapdoor_check must not be used on such params.
or_params *or_params_from_queries(const or_r1cs *cs, const uint8_t *h, uint64_t n_h, const uint8_t *l,
                                  const uint8_t *a, uint64_t n_a, const uint8_t *b_g1, const uint8_t *b_g2,
                                  uint64_t n_b, const uint8_t *vk, const uint8_t *ic) {
    or_params *P = new or_params();
    P->n = cs->num_constraints;
    P->n_in = cs->num_inputs;
    P->n_aux = cs->num_aux;
    P->log_d = domain_log(P->n + P->n_in);
    P->d = 1ULL << P->log_d;
    if (n_h != P->d - 1) {
        delete P;
        return nullptr;
    }
    P->a_aux_density.assign(P->n_aux, 0);
    P->b_in_density.assign(P->n_in, 0);
    P->b_aux_density.assign(P->n_aux, 0);
    for (int m = 0; m < 2; m++)
        for (uint64_t e = 0; e < cs->row_ptr[m][P->n]; e++) {
            uint32_t v = cs->col[m][e];
            if (m == 0 && v >= P->n_in) P->a_aux_density[v - P->n_in] = 1;
            if (m == 1) {
                if (v < P->n_in)
                    P->b_in_density[v] = 1;
                else
                    P->b_aux_density[v - P->n_in] = 1;
            }
        }
    P->h.resize(n_h);
    P->l.resize(P->n_aux);
    P->a.resize(n_a);
    P->b_g1.resize(n_b);
    P->b_g2.resize(n_b);
    P->ic.resize(P->n_in);
    bool ok = true;
    int nt = nthreads();
#pragma omp parallel for num_threads(nt) reduction(&& : ok)
    for (int64_t i = 0; i < (int64_t)n_h; i++) ok = ok && g1_decode(h + 96 * i, &P->h[i]);
#pragma omp parallel for num_threads(nt) reduction(&& : ok)
    for (int64_t i = 0; i < (int64_t)P->n_aux; i++) ok = ok && g1_decode(l + 96 * i, &P->l[i]);
#pragma omp parallel for num_threads(nt) reduction(&& : ok)
    for (int64_t i = 0; i < (int64_t)n_a; i++) ok = ok && g1_decode(a + 96 * i, &P->a[i]);
#pragma omp parallel for num_threads(nt) reduction(&& : ok)
    for (int64_t i = 0; i < (int64_t)n_b; i++)
        ok = ok && g1_decode(b_g1 + 96 * i, &P->b_g1[i]) && g2_decode(b_g2 + 192 * i, &P->b_g2[i]);
    for (uint64_t i = 0; i < P->n_in; i++) ok = ok && g1_decode(ic + 96 * i, &P->ic[i]);
    ok = ok && g1_decode(vk, &P->alpha_g1) && g1_decode(vk + 96, &P->beta_g1) && g2_decode(vk + 192, &P->beta_g2) &&
         g2_decode(vk + 384, &P->gamma_g2) && g1_decode(vk + 576, &P->delta_g1) && g2_decode(vk + 672, &P->delta_g2);
    if (!ok) {
        delete P;
        return nullptr;
    }
    return P;
}

void or_params_free(or_params *p) { delete p; }
void or_params_sizes(const or_params *p, uint64_t out[6]) {
    out[0] = p->d;
    out[1] = p->h.size();
    out[2] = p->l.size();
    out[3] = p->a.size();
    out[4] = p->b_g1.size();
    out[5] = p->b_g2.size();
}
void or_params_export(const or_params *p, uint8_t *h, uint8_t *l, uint8_t *a, uint8_t *b_g1, uint8_t *b_g2,
                      uint8_t *vk, uint8_t *ic) {
    if (h)
        for (size_t i = 0; i < p->h.size(); i++) g1_encode(p->h[i], h + 96 * i);
    if (l)
        for (size_t i = 0; i < p->l.size(); i++) g1_encode(p->l[i], l + 96 * i);
    if (a)
        for (size_t i = 0; i < p->a.size(); i++) g1_encode(p->a[i], a + 96 * i);
    if (b_g1)
        for (size_t i = 0; i < p->b_g1.size(); i++) g1_encode(p->b_g1[i], b_g1 + 96 * i);
    if (b_g2)
        for (size_t i = 0; i < p->b_g2.size(); i++) g2_encode(p->b_g2[i], b_g2 + 192 * i);
    if (vk) {
        g1_encode(p->alpha_g1, vk);
        g1_encode(p->beta_g1, vk + 96);
        g2_encode(p->beta_g2, vk + 192);
        g2_encode(p->gamma_g2, vk + 384);
        g1_encode(p->delta_g1, vk + 576);
        g2_encode(p->delta_g2, vk + 672);
    }
    if (ic)
        for (size_t i = 0; i < p->ic.size(); i++) g1_encode(p->ic[i], ic + 96 * i);
}

// bellman groth16::create_proof (with injected r, s)
int or_groth16_prove(const or_params *P, const or_r1cs *cs, const uint8_t *z32, const uint8_t r32[32],
                     const uint8_t s32[32], uint8_t proof_out[192], uint8_t *raw_out, uint8_t *h_out) {
    std::vector<fr> z = load_z(cs, z32);
    uint64_t d = P->d, n = P->n;
    std::vector<fr> a(d, FR::zero()), b(d, FR::zero()), c(d, FR::zero());
    int nt = nthreads();
#pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t j = 0; j < (int64_t)n; j++) {
        a[j] = lc_eval(cs, 0, j, z);
        b[j] = lc_eval(cs, 1, j, z);
        c[j] = lc_eval(cs, 2, j, z);
    }
    for (uint64_t i = 0; i < P->n_in; i++) a[n + i] = z[i];
    domain_op(a, P->log_d, 1);
    domain_op(a, P->log_d, 2);
    domain_op(b, P->log_d, 1);
    domain_op(b, P->log_d, 2);
    domain_op(c, P->log_d, 1);
    domain_op(c, P->log_d, 2);
    // divide_by_z_on_coset: Z(g w^i) = g^d - 1
    fr g = fr_from_u64(7);
    fr zinv = FR::inv(FR::sub(fr_pow_u64(g, d), FR::one()));
#pragma omp parallel for num_threads(nt)
    for (int64_t i = 0; i < (int64_t)d; i++) a[i] = FR::mul(FR::sub(FR::mul(a[i], b[i]), c[i]), zinv);
    domain_op(a, P->log_d, 3);
    // scalars (canonical)
    std::vector<uint64_t> hk(4 * (d - 1));
    for (uint64_t i = 0; i + 1 < d; i++) FR::to_raw(a[i], &hk[4 * i]);
    if (h_out)
        for (uint64_t i = 0; i + 1 < d; i++) memcpy(h_out + 32 * i, &hk[4 * i], 32);
    std::vector<uint64_t> zr(4 * z.size());
    for (size_t i = 0; i < z.size(); i++) FR::to_raw(z[i], &zr[4 * i]);
    typedef const uint64_t(*K)[4];
    g1j H = pippenger<G1>(P->h.data(), (K)hk.data(), d - 1);
    g1j L = pippenger<G1>(P->l.data(), (K)&zr[4 * P->n_in], P->n_aux);
    // A: inputs (full density) + aux (a_aux_density)
    std::vector<uint64_t> ka;
    for (uint64_t i = 0; i < P->n_in; i++) ka.insert(ka.end(), &zr[4 * i], &zr[4 * i + 4]);
    for (uint64_t i = 0; i < P->n_aux; i++)
        if (P->a_aux_density[i]) ka.insert(ka.end(), &zr[4 * (P->n_in + i)], &zr[4 * (P->n_in + i) + 4]);
    if (ka.size() / 4 != P->a.size()) return -2;
    std::vector<uint64_t> kb;
    for (uint64_t i = 0; i < P->n_in; i++)
        if (P->b_in_density[i]) kb.insert(kb.end(), &zr[4 * i], &zr[4 * i + 4]);
    for (uint64_t i = 0; i < P->n_aux; i++)
        if (P->b_aux_density[i]) kb.insert(kb.end(), &zr[4 * (P->n_in + i)], &zr[4 * (P->n_in + i) + 4]);
    if (kb.size() / 4 != P->b_g1.size()) return -3;
    g1j Asum = pippenger<G1>(P->a.data(), (K)ka.data(), P->a.size());
    g1j B1sum = pippenger<G1>(P->b_g1.data(), (K)kb.data(), P->b_g1.size());
    g2j B2sum = pippenger<G2>(P->b_g2.data(), (K)kb.data(), P->b_g2.size());
    uint64_t r[4], s[4], rs[4];
    memcpy(r, r32, 32);
    memcpy(s, s32, 32);
    fr rf = fr_from_le(r32), sf = fr_from_le(s32);
    FR::to_raw(FR::mul(rf, sf), rs);
    // A = alpha + sum_a + r delta
    g1j A = G1::add(G1::add(G1::from_aff(P->alpha_g1), Asum), G1::mul(G1::from_aff(P->delta_g1), r, 4));
    // B = beta + sum_b2 + s delta
    g2j B = G2::add(G2::add(G2::from_aff(P->beta_g2), B2sum), G2::mul(G2::from_aff(P->delta_g2), s, 4));
    // C = rs delta + s alpha + r beta + s sum_a + r sum_b1 + H + L
    g1j C = G1::mul(G1::from_aff(P->delta_g1), rs, 4);
    C = G1::add(C, G1::mul(G1::from_aff(P->alpha_g1), s, 4));
    C = G1::add(C, G1::mul(G1::from_aff(P->beta_g1), r, 4));
    C = G1::add(C, G1::mul(Asum, s, 4));
    C = G1::add(C, G1::mul(B1sum, r, 4));
    C = G1::add(C, H);
    C = G1::add(C, L);
    g1a Aa = G1::to_aff(A), Ca = G1::to_aff(C);
    g2a Ba = G2::to_aff(B);
    g1_compress(Aa, proof_out);
    g2_compress(Ba, proof_out + 48);
    g1_compress(Ca, proof_out + 144);
    if (raw_out) {
        g1_encode(Aa, raw_out);
        g2_encode(Ba, raw_out + 96);
        g1_encode(Ca, raw_out + 288);
    }
    return 0;
}

int or_groth16_trapdoor_check(const or_params *P, const or_r1cs *cs, const uint8_t *z32, const uint8_t r32[32],
                              const uint8_t s32[32], const uint8_t raw[384]) {
    std::vector<fr> z = load_z(cs, z32);
    fr u = FR::zero(), v = FR::zero(), w = FR::zero(), lsum = FR::zero();
    fr delta_inv = FR::inv(P->delta);
    for (size_t i = 0; i < z.size(); i++) {
        u = FR::add(u, FR::mul(z[i], P->at[i]));
        v = FR::add(v, FR::mul(z[i], P->bt[i]));
        w = FR::add(w, FR::mul(z[i], P->ct[i]));
        if (i >= P->n_in) {
            fr ext = FR::add(FR::add(FR::mul(P->beta, P->at[i]), FR::mul(P->alpha, P->bt[i])), P->ct[i]);
            lsum = FR::add(lsum, FR::mul(z[i], ext));
        }
    }
    fr rf = fr_from_le(r32), sf = fr_from_le(s32);
    fr Ad = FR::add(FR::add(P->alpha, u), FR::mul(rf, P->delta));
    fr Bd = FR::add(FR::add(P->beta, v), FR::mul(sf, P->delta));
    // h(tau) t(tau) = u v - w  (QAP identity for a satisfying witness)
    fr ht = FR::sub(FR::mul(u, v), w);
    fr Cd = FR::mul(FR::add(lsum, ht), delta_inv);
    Cd = FR::add(Cd, FR::mul(sf, Ad));
    Cd = FR::add(Cd, FR::mul(rf, Bd));
    Cd = FR::sub(Cd, FR::mul(FR::mul(rf, sf), P->delta));
    uint64_t ka[4], kb[4], kc[4];
    FR::to_raw(Ad, ka);
    FR::to_raw(Bd, kb);
    FR::to_raw(Cd, kc);
    g1a A, C;
    g2a B;
    if (!g1_decode(raw, &A) || !g2_decode(raw + 96, &B) || !g1_decode(raw + 288, &C)) return 0;
    g1j g1 = G1::from_aff(g1_gen());
    g2j g2 = G2::from_aff(g2_gen());
    bool ok = G1::eq(G1::from_aff(A), G1::mul(g1, ka, 4)) && G2::eq(G2::from_aff(B), G2::mul(g2, kb, 4)) &&
              G1::eq(G1::from_aff(C), G1::mul(g1, kc, 4));
    return ok ? 1 : 0;
}

int or_groth16_verify(const uint8_t vk[864], const uint8_t *ic96, uint64_t num_inputs, const uint8_t *inputs32,
                      const uint8_t raw[384]) {
    g1a alpha1, beta1, delta1, A, C;
    g2a beta2, gamma2, delta2, B;
    if (!g1_decode(vk, &alpha1) || !g1_decode(vk + 96, &beta1) || !g2_decode(vk + 192, &beta2) ||
        !g2_decode(vk + 384, &gamma2) || !g1_decode(vk + 576, &delta1) || !g2_decode(vk + 672, &delta2))
        return -1;
    if (!g1_decode(raw, &A) || !g2_decode(raw + 96, &B) || !g1_decode(raw + 288, &C)) return -1;
    if (!g1_on_curve(A) || !g2_on_curve(B) || !g1_on_curve(C)) return 0;
    // IC = sum inputs_i * ic_i
    g1j IC = G1::identity();
    for (uint64_t i = 0; i < num_inputs; i++) {
        g1a p;
        if (!g1_decode(ic96 + 96 * i, &p)) return -1;
        uint64_t k[4];
        memcpy(k, inputs32 + 32 * i, 32);
        IC = G1::add(IC, G1::mul(G1::from_aff(p), k, 4));
    }
    g1a ICa = G1::to_aff(IC);
    // e(A,B) == e(alpha,beta) e(IC,gamma) e(C,delta)  <=>  ML(A,B) ML(-alpha,beta) ML(-IC,gamma) ML(-C,delta) ^ fe == 1
    fq12 f = miller_loop(B, A);
    f = f12_mul(f, miller_loop(beta2, G1::neg(alpha1)));
    f = f12_mul(f, miller_loop(gamma2, G1::neg(ICa)));
    f = f12_mul(f, miller_loop(delta2, G1::neg(C)));
    fq12 e = f12_pow_big(f, final_exponent());
    return f12_eq(e, f12_one()) ? 1 : 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------------
// SDR labelling witness: SHA-256 (FIPS 180-4, restated) and the stacked-DRG label
//   label = SHA256(replica_id || u32_be(layer) || u64_be(node) || 0^20 || parents[0..P_full)) with the
//   top two bits of byte 31 cleared.  Follows LabelingProof create_label
//   (libs/storage/include/nil/filecoin/storage/proofs/porep/stacked/vanilla/detail/processing/naive/
//   labelling_proof.hpp:46-60), create_label (vanilla/create_label.hpp:43-78: the 32-byte prefix block
//   whose 12-byte truncation the reference shows, then the parents, "strip last two bits") and the cyclic
//   parent repetition to TOTAL_PARENTS = 37 (vanilla/proof.hpp:49, 233-237).  n_parents = 0 is node 0's
//   label (no parents: create_label.hpp:67-69).
namespace {
const uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

inline uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

void sha256_block(uint32_t h[8], const uint8_t *blk) {
    uint32_t w[64];
    for (int t = 0; t < 16; t++)
        w[t] = (uint32_t)blk[4 * t] << 24 | (uint32_t)blk[4 * t + 1] << 16 | (uint32_t)blk[4 * t + 2] << 8 | blk[4 * t + 3];
    for (int t = 16; t < 64; t++) {
        const uint32_t s0 = rotr32(w[t - 15], 7) ^ rotr32(w[t - 15], 18) ^ (w[t - 15] >> 3);
        const uint32_t s1 = rotr32(w[t - 2], 17) ^ rotr32(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
    for (int t = 0; t < 64; t++) {
        const uint32_t t1 = k + (rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25)) + ((e & f) ^ (~e & g)) + kSha256K[t] + w[t];
        const uint32_t t2 = (rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

// streaming SHA-256 over a message given as pieces
struct Sha256 {
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint8_t buf[64];
    size_t fill = 0;
    uint64_t len = 0;
    void update(const uint8_t *p, size_t n) {
        len += n;
        while (n) {
            const size_t take = std::min(n, 64 - fill);
            memcpy(buf + fill, p, take);
            fill += take; p += take; n -= take;
            if (fill == 64) { sha256_block(h, buf); fill = 0; }
        }
    }
    void finish(uint8_t out[32]) {
        const uint64_t bits = len * 8;
        const uint8_t pad = 0x80, zero = 0;
        update(&pad, 1);
        while (fill != 56) update(&zero, 1);
        uint8_t l[8];
        for (int i = 0; i < 8; i++) l[i] = (uint8_t)(bits >> (56 - 8 * i));
        update(l, 8);
        for (int i = 0; i < 8; i++)
            for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(h[i] >> (24 - 8 * j));
    }
};
}  // namespace

extern "C" {
void or_sha256(const uint8_t *msg, uint64_t len, uint8_t out[32]) {
    Sha256 s;
    s.update(msg, len);
    s.finish(out);
}

int or_sdr_labels(const uint8_t replica_id[32], uint64_t count, const uint32_t *layers, const uint64_t *nodes,
                  const uint8_t *parents, unsigned n_parents, uint8_t *labels) {
    if (n_parents > 37) return -1;
    const int nt = nthreads();
#pragma omp parallel for num_threads(nt) schedule(static) if (count >= 256)
    for (int64_t i = 0; i < (int64_t)count; i++) {
        uint8_t pre[64] = {0};
        memcpy(pre, replica_id, 32);
        for (int j = 0; j < 4; j++) pre[32 + j] = (uint8_t)(layers[i] >> (24 - 8 * j));
        for (int j = 0; j < 8; j++) pre[36 + j] = (uint8_t)(nodes[i] >> (56 - 8 * j));
        Sha256 s;
        s.update(pre, 64);
        const uint8_t *p = parents + (uint64_t)i * n_parents * 32;
        if (n_parents)
            for (unsigned k = 0; k < 37; k++) s.update(p + 32 * (k % n_parents), 32);
        uint8_t *o = labels + 32 * (uint64_t)i;
        s.finish(o);
        o[31] &= 0x3f;
    }
    return 0;
}
}  // extern "C"
