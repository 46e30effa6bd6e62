// hostfield.h -- host-only BLS12-381 Fq / Fq2 over 6 x 64-bit limbs (CIOS Montgomery, R = 2^384) for the serial
// group-law chains that run on the CPU: the MSM window combination (Horner over the windows, c doublings each)
// and the proof assembly's scalar multiplications by r, s and the blinding terms.
//
// The device field (field.h: 13 balanced 30-bit limbs) is shaped for wave64 v_mad_i64_i32 issue; compiled for the
// host it costs 338 64-bit multiplies per product.  Here a product is 36 64 x 64 -> 128 multiplies (x86 mulx
// through unsigned __int128), so the host chains run several times faster.  Values are canonical in [0, p).
// The group law is curve.h's (the same XYZZ formulas, instantiated over hfq / hfq2); values cross between the
// two representations through the canonical 12 x 32-bit integer (fq_to_raw / fq_from_raw).
#pragma once
#include <stdint.h>

#include <vector>

#include "curve.h"

namespace mi {
namespace host {

struct HP {
    static constexpr uint64_t P[6] = {0xb9feffffffffaaabull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull,
                                      0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
    static constexpr uint64_t INV = 0x89f3fffcfffcfffdull;  // -p^-1 mod 2^64
    static constexpr uint64_t ONE[6] = {0x760900000002fffdull, 0xebf4000bc40c0002ull, 0x5f48985753c758baull,
                                        0x77ce585370525745ull, 0x5c071a97a256ec6dull, 0x15f65ec3fa80e493ull};
    static constexpr uint64_t R2[6] = {0xf4df1f341c341746ull, 0x0a76e6a609d104f1ull, 0x8de5476c4c95b6d5ull,
                                       0x67eb88a9939d83c0ull, 0x9a793e85b519952dull, 0x11988fe592cae3aaull};
};

typedef unsigned __int128 u128;

struct hfq {
    uint64_t v[6];
    static hfq zero() { return {{0, 0, 0, 0, 0, 0}}; }
    static hfq one() {
        hfq r;
        for (int i = 0; i < 6; i++) r.v[i] = HP::ONE[i];
        return r;
    }
    bool is_zero() const { return (v[0] | v[1] | v[2] | v[3] | v[4] | v[5]) == 0; }
    bool operator==(const hfq &o) const {
        uint64_t x = 0;
        for (int i = 0; i < 6; i++) x |= v[i] ^ o.v[i];
        return x == 0;
    }
    bool operator!=(const hfq &o) const { return !(*this == o); }
};

inline hfq hfq_sub_p_if_ge(const uint64_t t[6], uint64_t hi) {  // t (+ hi 2^384) < 2p -> t mod p
    hfq r;
    uint64_t bw = 0;
    for (int i = 0; i < 6; i++) {
        const u128 d = (u128)t[i] - HP::P[i] - bw;
        r.v[i] = (uint64_t)d;
        bw = (uint64_t)(d >> 64) & 1;
    }
    const uint64_t keep = (uint64_t)0 - (uint64_t)(bw > hi);  // t < p: keep t
    for (int i = 0; i < 6; i++) r.v[i] = (t[i] & keep) | (r.v[i] & ~keep);
    return r;
}

inline hfq operator+(const hfq &a, const hfq &b) {
    uint64_t t[6], c = 0;
    for (int i = 0; i < 6; i++) {
        const u128 s = (u128)a.v[i] + b.v[i] + c;
        t[i] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
    }
    return hfq_sub_p_if_ge(t, c);
}
inline hfq operator-(const hfq &a, const hfq &b) {
    hfq r;
    uint64_t bw = 0;
    for (int i = 0; i < 6; i++) {
        const u128 d = (u128)a.v[i] - b.v[i] - bw;
        r.v[i] = (uint64_t)d;
        bw = (uint64_t)(d >> 64) & 1;
    }
    if (bw) {
        uint64_t c = 0;
        for (int i = 0; i < 6; i++) {
            const u128 s = (u128)r.v[i] + HP::P[i] + c;
            r.v[i] = (uint64_t)s;
            c = (uint64_t)(s >> 64);
        }
    }
    return r;
}
inline hfq operator-(const hfq &a) { return hfq::zero() - a; }
inline hfq dbl(const hfq &a) { return a + a; }

// CIOS Montgomery product a b 2^-384 mod p.  p < 2^382 leaves the top word two spare bits, so the running
// total never needs a seventh word (the "no-carry" CIOS form: the product and the reduction of each outer
// step share one inner loop); the result is < 2p and one branchless subtraction makes it canonical.
inline hfq operator*(const hfq &a, const hfq &b) {
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 6; i++) {
        u128 s = (u128)a.v[0] * b.v[i] + t[0];
        uint64_t A = (uint64_t)(s >> 64);
        const uint64_t m = (uint64_t)s * HP::INV;
        u128 q = (u128)m * HP::P[0] + (uint64_t)s;
        uint64_t C = (uint64_t)(q >> 64);
        for (int j = 1; j < 6; j++) {
            s = (u128)a.v[j] * b.v[i] + t[j] + A;
            A = (uint64_t)(s >> 64);
            q = (u128)m * HP::P[j] + (uint64_t)s + C;
            C = (uint64_t)(q >> 64);
            t[j - 1] = (uint64_t)q;
        }
        t[5] = A + C;
    }
    return hfq_sub_p_if_ge(t, 0);
}
inline hfq sqr(const hfq &a) { return a * a; }
inline hfq mul_add(const hfq &a, const hfq &b, const hfq &c, const hfq &d) { return a * b + c * d; }
inline hfq inverse_inl(const hfq &a) {  // a^(p - 2)
    static const uint64_t E[6] = {0xb9feffffffffaaa9ull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull,
                                  0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
    hfq r = hfq::one();
    for (int i = 5; i >= 0; i--)
        for (int b = 63; b >= 0; b--) {
            r = r * r;
            if ((E[i] >> b) & 1) r = r * a;
        }
    return r;
}

struct hfq2 {
    hfq c0, c1;
    static hfq2 zero() { return {hfq::zero(), hfq::zero()}; }
    static hfq2 one() { return {hfq::one(), hfq::zero()}; }
    bool is_zero() const { return c0.is_zero() && c1.is_zero(); }
    bool operator==(const hfq2 &o) const { return c0 == o.c0 && c1 == o.c1; }
    bool operator!=(const hfq2 &o) const { return !(*this == o); }
};
inline hfq2 operator+(const hfq2 &a, const hfq2 &b) { return {a.c0 + b.c0, a.c1 + b.c1}; }
inline hfq2 operator-(const hfq2 &a, const hfq2 &b) { return {a.c0 - b.c0, a.c1 - b.c1}; }
inline hfq2 operator-(const hfq2 &a) { return {-a.c0, -a.c1}; }
inline hfq2 dbl(const hfq2 &a) { return a + a; }
inline hfq2 operator*(const hfq2 &a, const hfq2 &b) {  // Karatsuba over u^2 = -1
    const hfq v0 = a.c0 * b.c0, v1 = a.c1 * b.c1;
    return {v0 - v1, (a.c0 + a.c1) * (b.c0 + b.c1) - v0 - v1};
}
inline hfq2 sqr(const hfq2 &a) {
    const hfq t = a.c0 * a.c1;
    return {(a.c0 + a.c1) * (a.c0 - a.c1), t + t};
}
inline hfq2 mul_add(const hfq2 &a, const hfq2 &b, const hfq2 &c, const hfq2 &d) { return a * b + c * d; }
inline hfq2 inverse_inl(const hfq2 &a) {
    const hfq n = inverse_inl(sqr(a.c0) + sqr(a.c1));
    return {a.c0 * n, -(a.c1 * n)};
}

// ---- conversions through the canonical integer ----
inline hfq to_h(const fq_t &a) {
    const fq32_t raw = fq_to_raw(a);
    hfq x;
    for (int i = 0; i < 6; i++) x.v[i] = (uint64_t)raw.v[2 * i] | ((uint64_t)raw.v[2 * i + 1] << 32);
    hfq r2;
    for (int i = 0; i < 6; i++) r2.v[i] = HP::R2[i];
    return x * r2;
}
inline fq_t from_h(const hfq &a) {
    hfq one_raw = hfq::zero();
    one_raw.v[0] = 1;
    const hfq x = a * one_raw;
    fq32_t raw;
    for (int i = 0; i < 6; i++) {
        raw.v[2 * i] = (uint32_t)x.v[i];
        raw.v[2 * i + 1] = (uint32_t)(x.v[i] >> 32);
    }
    return fq_from_raw(raw);
}
inline hfq2 to_h(const fq2_t &a) { return {to_h(a.c0), to_h(a.c1)}; }
inline fq2_t from_h(const hfq2 &a) { return {from_h(a.c0), from_h(a.c1)}; }

template <class F>
struct HostOf;
template <>
struct HostOf<fq_t> {
    using T = hfq;
};
template <>
struct HostOf<fq2_t> {
    using T = hfq2;
};

template <class F>
XYZZ<typename HostOf<F>::T> to_h(const XYZZ<F> &p) {
    if (p.is_inf()) return XYZZ<typename HostOf<F>::T>::inf();
    return {to_h(p.X), to_h(p.Y), to_h(p.ZZ), to_h(p.ZZZ)};
}
template <class F>
XYZZ<F> from_h(const XYZZ<typename HostOf<F>::T> &p) {
    if (p.is_inf()) return XYZZ<F>::inf();
    return {from_h(p.X), from_h(p.Y), from_h(p.ZZ), from_h(p.ZZZ)};
}

// ---- the host chains ----
// k P (k: little-endian 32-bit words), the scalar multiplication of the proof assembly and key generation
template <class F>
XYZZ<F> xyzz_mul(const XYZZ<F> &p, const uint32_t *k, int nwords) {
    return from_h<F>(mi::xyzz_mul_inl(to_h(p), k, nwords));
}
template <class F>
XYZZ<F> xyzz_add(const XYZZ<F> &p, const XYZZ<F> &q) {
    return from_h<F>(mi::xyzz_add_inl(to_h(p), to_h(q)));
}
template <class F>
XYZZ<F> xyzz_add_affine(const XYZZ<F> &p, const Affine<F> &q) {
    if (q.is_inf()) return p;
    return from_h<F>(mi::xyzz_add_inl(to_h(p), to_h(xyzz_from_affine(q))));
}
template <class F>
Affine<F> xyzz_to_affine(const XYZZ<F> &p) {
    if (p.is_inf()) return Affine<F>::inf();
    const auto a = mi::xyzz_to_affine_inl(to_h(p));
    return {from_h(a.x), from_h(a.y)};
}
// 2^n p
template <class F>
XYZZ<F> xyzz_dbl_n(const XYZZ<F> &p, unsigned n) {
    if (n == 0 || p.is_inf()) return p;
    auto t = to_h(p);
    for (unsigned i = 0; i < n; i++) t = mi::xyzz_dbl_inl(t);
    return from_h<F>(t);
}
// sum_w 2^(c w) W[w] by Horner over the windows (c doublings per window): the MSM's final combination
template <class F>
XYZZ<F> combine_windows(const std::vector<XYZZ<F>> &W, unsigned c) {
    using H = typename HostOf<F>::T;
    if (W.empty()) return XYZZ<F>::inf();
    XYZZ<H> acc = to_h(W.back());
    for (int w = (int)W.size() - 2; w >= 0; w--) {
        for (unsigned i = 0; i < c; i++) acc = mi::xyzz_dbl_inl(acc);
        acc = mi::xyzz_add_inl(acc, to_h(W[w]));
    }
    return from_h<F>(acc);
}
// SumA + 2^s (V - R) per window (reduce_windows' recombination of its two running-sum levels)
template <class F>
XYZZ<F> window_from_sums(const XYZZ<F> &sum_a, const XYZZ<F> &r, const XYZZ<F> &v, unsigned log_seg) {
    using H = typename HostOf<F>::T;
    XYZZ<H> t = mi::xyzz_add_inl(to_h(v), mi::xyzz_neg(to_h(r)));
    for (unsigned i = 0; i < log_seg; i++) t = mi::xyzz_dbl_inl(t);
    return from_h<F>(mi::xyzz_add_inl(to_h(sum_a), t));
}

}  // namespace host
}  // namespace mi
