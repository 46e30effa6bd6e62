// fr29.h -- Fr (BLS12-381 scalar field) over 9 x 29-bit limbs, Montgomery radix R = 2^261 (the radix of
// fr_t, so converting is repacking): the in-register representation of the Poseidon permutation and the
// NTT passes.  Values are kept lazily below a small multiple of r: REDC(a b) < a b / R + r, and
// r / R < 2^-6, so operands up to ~8r give products below 2r; the column-sum bound of the product
// scanning only needs carry-normalised 29-bit limbs.
#pragma once
#include "field.h"

namespace mi {

// Fr in 9 x 29-bit limbs; 8-byte aligned (40 bytes) so vectorised copies never straddle two elements
struct alignas(8) fr29_t {
    uint32_t v[9];
};

constexpr uint32_t M29 = (1u << 29) - 1;
// 2r in 29-bit limbs (conditional subtraction), r itself is FrDesc::MOD29
constexpr uint32_t R2X29[9] = {0x00000002u, 0x1ffffff0u, 0x1f2dff7fu, 0x16900bffu, 0x1b00aa77u,
                               0x180809a1u, 0x0a4199ceu, 0x14ca675fu, 0x00e7db4eu};

MI_HD fr29_t fr29_from_fr(const fr_t &a) {
    fr29_t r;
    MI_UNROLL for (int i = 0; i < 9; i++) {
        const int bit = 29 * i, w = bit >> 5, s = bit & 31;
        uint64_t x = a.v[w];
        if (w + 1 < 8) x |= (uint64_t)a.v[w + 1] << 32;
        r.v[i] = (uint32_t)(x >> s) & M29;
    }
    return r;
}
// value < 2^256 (canonical here)
MI_HD fr_t fr_from_fr29(const fr29_t &t) {
    fr_t r;
    MI_UNROLL for (int j = 0; j < 8; j++) r.v[j] = 0;
    MI_UNROLL for (int i = 0; i < 9; i++) {
        const int bit = 29 * i, w = bit >> 5, s = bit & 31;
        r.v[w] |= t.v[i] << s;
        if (s > 3 && w + 1 < 8) r.v[w + 1] |= t.v[i] >> (32 - s);
    }
    return r;
}

// sum_k a[k] b[k] R^-1 with one Montgomery reduction, K <= 6 (column sums <= 63 products < 2^58 plus a
// carry < 2^35 stay below 2^64).  Result < sum a_k b_k / R + r.
template <int K>
MI_HD fr29_t fr29_dot(const fr29_t *a, const fr29_t *b) {
    static_assert(K >= 1 && K <= 6, "fr29_dot: at most 6 products per reduction");
    constexpr int L = 9;
    uint32_t m[L];
    fr29_t r;
    uint64_t acc = 0;
    MI_UNROLL for (int k = 0; k < L; k++) {
        MI_UNROLL for (int i = 0; i < k; i++) {
            MI_UNROLL for (int q = 0; q < K; q++) acc += (uint64_t)a[q].v[i] * b[q].v[k - i];
            acc += (uint64_t)m[i] * FrDesc::MOD29[k - i];
        }
        MI_UNROLL for (int q = 0; q < K; q++) acc += (uint64_t)a[q].v[k] * b[q].v[0];
        m[k] = ((uint32_t)acc * FrDesc::INV29) & M29;
        acc += (uint64_t)m[k] * FrDesc::MOD29[0];
        acc >>= 29;
    }
    MI_UNROLL for (int k = L; k < 2 * L - 1; k++) {
        MI_UNROLL for (int i = k - L + 1; i < L; i++) {
            MI_UNROLL for (int q = 0; q < K; q++) acc += (uint64_t)a[q].v[i] * b[q].v[k - i];
            acc += (uint64_t)m[i] * FrDesc::MOD29[k - i];
        }
        r.v[k - L] = (uint32_t)acc & M29;
        acc >>= 29;
    }
    r.v[L - 1] = (uint32_t)acc;
    return r;
}
MI_HD fr29_t fr29_mul(const fr29_t &a, const fr29_t &b) { return fr29_dot<1>(&a, &b); }

// a + b, carry-normalised, not reduced
MI_HD fr29_t fr29_add(const fr29_t &a, const fr29_t &b) {
    fr29_t r;
    uint32_t c = 0;
    MI_UNROLL for (int i = 0; i < 8; i++) {
        uint32_t t = a.v[i] + b.v[i] + c;
        r.v[i] = t & M29;
        c = t >> 29;
    }
    r.v[8] = a.v[8] + b.v[8] + c;
    return r;
}
// a - m if a >= m, for m = r or 2r given in 29-bit limbs
MI_HD fr29_t fr29_sub_if_ge(const fr29_t &a, const uint32_t *m) {
    fr29_t d;
    int32_t bw = 0;
    MI_UNROLL for (int i = 0; i < 8; i++) {
        int32_t t = (int32_t)a.v[i] - (int32_t)m[i] + bw;
        d.v[i] = (uint32_t)t & M29;
        bw = t >> 29;
    }
    const int32_t top = (int32_t)a.v[8] - (int32_t)m[8] + bw;
    d.v[8] = (uint32_t)top;
    return top < 0 ? a : d;
}
// x^2 over the symmetric products only ((2 a_i) a_(k-i), i < k - i, and a_(k/2)^2): 45 + 81 MADs instead
// of 81 + 81.  2 a_i fits 32 bits for operands below 2^31 r, and the column sums stay within fr29_dot<1>'s.
MI_HD fr29_t fr29_sqr(const fr29_t &a) {
    constexpr int L = 9;
    uint32_t a2[L];
    MI_UNROLL for (int i = 0; i < L; i++) a2[i] = a.v[i] << 1;
    uint32_t m[L];
    fr29_t r;
    uint64_t acc = 0;
    MI_UNROLL for (int k = 0; k < L; k++) {
        MI_UNROLL for (int i = 0; i < k - i; i++) acc += (uint64_t)a2[i] * a.v[k - i];
        if ((k & 1) == 0) acc += (uint64_t)a.v[k >> 1] * a.v[k >> 1];
        MI_UNROLL for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * FrDesc::MOD29[k - i];
        m[k] = ((uint32_t)acc * FrDesc::INV29) & M29;
        acc += (uint64_t)m[k] * FrDesc::MOD29[0];
        acc >>= 29;
    }
    MI_UNROLL for (int k = L; k < 2 * L - 1; k++) {
        MI_UNROLL for (int i = k - L + 1; i < k - i; i++) acc += (uint64_t)a2[i] * a.v[k - i];
        if ((k & 1) == 0) acc += (uint64_t)a.v[k >> 1] * a.v[k >> 1];
        MI_UNROLL for (int i = k - L + 1; i < L; i++) acc += (uint64_t)m[i] * FrDesc::MOD29[k - i];
        r.v[k - L] = (uint32_t)acc & M29;
        acc >>= 29;
    }
    r.v[L - 1] = (uint32_t)acc;
    return r;
}
MI_HD fr29_t fr29_sbox(const fr29_t &x) {  // x^5
    const fr29_t x2 = fr29_sqr(x);
    const fr29_t x4 = fr29_sqr(x2);
    return fr29_mul(x4, x);
}
// Montgomery value < 4r -> canonical integer < r
MI_HD fr29_t fr29_from_mont(const fr29_t &a) {
    fr29_t one = {{1, 0, 0, 0, 0, 0, 0, 0, 0}};
    return fr29_sub_if_ge(fr29_mul(a, one), FrDesc::MOD29);  // REDC(a) < a / R + r <= r
}


// a - b + k r for b < k r (k r given in 29-bit limbs): normalised, not reduced
MI_HD fr29_t fr29_sub_lazy(const fr29_t &a, const fr29_t &b, const uint32_t *kr) {
    fr29_t d;
    int32_t c = 0;
    MI_UNROLL for (int i = 0; i < 8; i++) {
        int32_t t = (int32_t)a.v[i] - (int32_t)b.v[i] + (int32_t)kr[i] + c;
        d.v[i] = (uint32_t)t & M29;
        c = t >> 29;
    }
    d.v[8] = (uint32_t)((int32_t)a.v[8] - (int32_t)b.v[8] + (int32_t)kr[8] + c);
    return d;
}

}  // namespace mi
