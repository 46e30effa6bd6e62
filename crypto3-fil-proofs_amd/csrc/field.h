// field.h -- BLS12-381 base field Fq (381-bit) and scalar field Fr (255-bit) in Montgomery form.
//
// Restates crypto3's multiprecision Montgomery backend ([NOT IN TREE]: libs/crypto/multiprecision,
// used via algebra::curves::bls12<381>, core/crypto/scheme_params.hpp:39-43) for CDNA4:
//   * Fq (the MSM hot loop) uses 14 limbs of 29 bits, Montgomery radix R = 2^406, product-scanning
//     (FIPS) Montgomery multiplication: a column holds <= 28 products < 2^58, so every limb product
//     is ONE v_mad_u64_u32 accumulating into a 64-bit register pair and carries move once per
//     column -- 544 instructions per multiplication vs 1453 for 32-bit CIOS, measured 79 vs 39
//     G Fq-mul/s on MI355X (microbench/fieldmul.hip).  Values are kept lazily in [0, 2p): the
//     product of two such values is again < 2p because R > 4p, so there is no final subtraction.
//   * Fr (NTT, scalars) uses 8 limbs of 32 bits with "no-carry" CIOS (top limb < 2^31 - 1); its
//     memory image is the canonical 32-byte little-endian encoding.
//   * everything is fully unrolled so elements live in VGPRs (Fq = 14, Fr = 8 registers).
// The same code compiles for the host (final window combination, proof assembly).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MI_HD __host__ __device__ __forceinline__
#define MI_UNROLL _Pragma("unroll")
// group-law level functions are compiled once and called (keeps kernels and build times small)
#define MI_NOINL __host__ __device__ __attribute__((noinline)) inline

namespace mi {

struct FqDesc {
    static constexpr int N = 12;
    static constexpr uint32_t INV = 0xfffcfffdu;  // -p^-1 mod 2^32
    static constexpr uint32_t MOD[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu,
                                         0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu, 0x64774b84u,
                                         0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
    static constexpr uint32_t R1[12] = {0x0002fffdu, 0x76090000u, 0xc40c0002u, 0xebf4000bu,
                                        0x53c758bau, 0x5f489857u, 0x70525745u, 0x77ce5853u,
                                        0xa256ec6du, 0x5c071a97u, 0xfa80e493u, 0x15f65ec3u};
    static constexpr uint32_t R2[12] = {0x1c341746u, 0xf4df1f34u, 0x09d104f1u, 0x0a76e6a6u,
                                        0x4c95b6d5u, 0x8de5476cu, 0x939d83c0u, 0x67eb88a9u,
                                        0xb519952du, 0x9a793e85u, 0x92cae3aau, 0x11988fe5u};
};

struct FrDesc {
    static constexpr int N = 8;
    static constexpr uint32_t INV = 0xffffffffu;  // r = 1 mod 2^32
    static constexpr uint32_t MOD[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                                        0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
    // Montgomery radix R = 2^261 (products are computed over 9 x 29-bit limbs, see operator*)
    static constexpr uint32_t R1[8] = {0xffffffbau, 0x00000045u, 0x0072d846u, 0x1a25272eu,
                                       0x5dbeee8bu, 0xfe2eedcdu, 0x9eefbe41u, 0x4d043f42u};
    static constexpr uint32_t R2[8] = {0xca71b3c0u, 0x67a6440fu, 0x49d98f66u, 0xc44e2d5eu,
                                       0xe8703b58u, 0x7ddc57c6u, 0x009cf20au, 0x27fd91b3u};
    static constexpr int L29 = 9;
    static constexpr uint32_t MOD29[9] = {0x00000001u, 0x1ffffff8u, 0x1f96ffbfu, 0x1b4805ffu, 0x1d80553bu,
                                          0x0c0404d0u, 0x1520cce7u, 0x0a6533afu, 0x0073eda7u};
    static constexpr uint32_t INV29 = 0x1fffffffu;  // -r^-1 mod 2^29
};

template <class D>
struct alignas(16) Fp {
    static constexpr int N = D::N;
    uint32_t v[D::N];

    MI_HD static Fp zero() {
        Fp r;
        MI_UNROLL for (int i = 0; i < N; i++) r.v[i] = 0;
        return r;
    }
    MI_HD static Fp one() {  // Montgomery 1 = R mod p
        Fp r;
        MI_UNROLL for (int i = 0; i < N; i++) r.v[i] = D::R1[i];
        return r;
    }
    MI_HD static Fp modulus_raw() {
        Fp r;
        MI_UNROLL for (int i = 0; i < N; i++) r.v[i] = D::MOD[i];
        return r;
    }
    MI_HD bool is_zero() const {
        uint32_t x = 0;
        MI_UNROLL for (int i = 0; i < N; i++) x |= v[i];
        return x == 0;
    }
    MI_HD bool operator==(const Fp &o) const {
        uint32_t x = 0;
        MI_UNROLL for (int i = 0; i < N; i++) x |= v[i] ^ o.v[i];
        return x == 0;
    }
    MI_HD bool operator!=(const Fp &o) const { return !(*this == o); }
};

// r = a - MOD if a >= MOD else a   (a < 2 MOD)
template <class D>
MI_HD Fp<D> reduce_once(const Fp<D> &a) {
    Fp<D> t;
    uint32_t borrow = 0;
    MI_UNROLL for (int i = 0; i < D::N; i++) {
        uint64_t d = (uint64_t)a.v[i] - D::MOD[i] - borrow;
        t.v[i] = (uint32_t)d;
        borrow = (uint32_t)(d >> 63);
    }
    return borrow ? a : t;
}

template <class D>
MI_HD Fp<D> operator+(const Fp<D> &a, const Fp<D> &b) {
    Fp<D> r;
    uint32_t carry = 0;
    MI_UNROLL for (int i = 0; i < D::N; i++) {
        uint64_t s = (uint64_t)a.v[i] + b.v[i] + carry;
        r.v[i] = (uint32_t)s;
        carry = (uint32_t)(s >> 32);
    }
    // both moduli leave >= 1 spare top bit, so a + b < 2^(32N) and carry is always 0
    return reduce_once(r);
}

template <class D>
MI_HD Fp<D> operator-(const Fp<D> &a, const Fp<D> &b) {
    Fp<D> r;
    uint32_t borrow = 0;
    MI_UNROLL for (int i = 0; i < D::N; i++) {
        uint64_t d = (uint64_t)a.v[i] - b.v[i] - borrow;
        r.v[i] = (uint32_t)d;
        borrow = (uint32_t)(d >> 63);
    }
    if (borrow) {
        uint32_t carry = 0;
        MI_UNROLL for (int i = 0; i < D::N; i++) {
            uint64_t s = (uint64_t)r.v[i] + D::MOD[i] + carry;
            r.v[i] = (uint32_t)s;
            carry = (uint32_t)(s >> 32);
        }
    }
    return r;
}

template <class D>
MI_HD Fp<D> operator-(const Fp<D> &a) {
    return Fp<D>::zero() - a;
}

template <class D>
MI_HD Fp<D> dbl(const Fp<D> &a) {
    return a + a;
}

// No-carry CIOS Montgomery multiplication: a * b * 2^(-32N) mod p.
template <class D>
MI_HD Fp<D> operator*(const Fp<D> &a, const Fp<D> &b) {
    constexpr int N = D::N;
    uint32_t t[N];
    MI_UNROLL for (int j = 0; j < N; j++) t[j] = 0;
    MI_UNROLL for (int i = 0; i < N; i++) {
        uint64_t p = (uint64_t)a.v[0] * b.v[i] + t[0];
        uint32_t A = (uint32_t)(p >> 32);
        uint32_t t0 = (uint32_t)p;
        uint32_t m = t0 * D::INV;
        uint64_t q = (uint64_t)m * D::MOD[0] + t0;
        uint32_t C = (uint32_t)(q >> 32);
        MI_UNROLL for (int j = 1; j < N; j++) {
            p = (uint64_t)a.v[j] * b.v[i] + t[j] + A;
            A = (uint32_t)(p >> 32);
            q = (uint64_t)m * D::MOD[j] + (uint32_t)p + C;
            C = (uint32_t)(q >> 32);
            t[j - 1] = (uint32_t)q;
        }
        t[N - 1] = C + A;
    }
    Fp<D> r;
    MI_UNROLL for (int j = 0; j < N; j++) r.v[j] = t[j];
    return reduce_once(r);
}

// Fr: storage stays 8 x 32-bit (canonical Montgomery value < r, the wire/memory image), but the
// product is computed by product scanning over 9 x 29-bit limbs (R = 2^261): 162 v_mad_u64_u32 and
// no carry chains instead of the 32-bit CIOS above; result < 2r, one conditional subtraction.
template <>
MI_HD Fp<FrDesc> operator*<FrDesc>(const Fp<FrDesc> &a, const Fp<FrDesc> &b) {
    constexpr int L = 9;
    constexpr uint32_t M = (1u << 29) - 1;
    uint32_t x[L], y[L], m[L], t[L];
    MI_UNROLL for (int i = 0; i < L; i++) {
        const int bit = 29 * i, w = bit >> 5, s = bit & 31;
        uint64_t xa = a.v[w], xb = b.v[w];
        if (w + 1 < 8) {
            xa |= (uint64_t)a.v[w + 1] << 32;
            xb |= (uint64_t)b.v[w + 1] << 32;
        }
        x[i] = (uint32_t)(xa >> s) & M;
        y[i] = (uint32_t)(xb >> s) & M;
    }
    uint64_t acc = 0;
    MI_UNROLL for (int k = 0; k < L; k++) {
        MI_UNROLL for (int i = 0; i < k; i++) {
            acc += (uint64_t)x[i] * y[k - i];
            acc += (uint64_t)m[i] * FrDesc::MOD29[k - i];
        }
        acc += (uint64_t)x[k] * y[0];
        m[k] = ((uint32_t)acc * FrDesc::INV29) & M;
        acc += (uint64_t)m[k] * FrDesc::MOD29[0];
        acc >>= 29;
    }
    MI_UNROLL for (int k = L; k < 2 * L - 1; k++) {
        MI_UNROLL for (int i = k - L + 1; i < L; i++) {
            acc += (uint64_t)x[i] * y[k - i];
            acc += (uint64_t)m[i] * FrDesc::MOD29[k - i];
        }
        t[k - L] = (uint32_t)acc & M;
        acc >>= 29;
    }
    t[L - 1] = (uint32_t)acc;
    Fp<FrDesc> r;
    MI_UNROLL for (int j = 0; j < 8; j++) r.v[j] = 0;
    MI_UNROLL for (int i = 0; i < L; i++) {
        const int bit = 29 * i, w = bit >> 5, s = bit & 31;
        r.v[w] |= t[i] << s;
        if (s > 3 && w + 1 < 8) r.v[w + 1] |= t[i] >> (32 - s);
    }
    return reduce_once(r);
}

template <class D>
MI_HD Fp<D> sqr(const Fp<D> &a) {
    return a * a;
}

// canonical (raw integer < p) -> Montgomery
template <class D>
MI_HD Fp<D> to_mont(const Fp<D> &raw) {
    Fp<D> r2;
    MI_UNROLL for (int i = 0; i < D::N; i++) r2.v[i] = D::R2[i];
    return raw * r2;
}
// Montgomery -> canonical
template <class D>
MI_HD Fp<D> from_mont(const Fp<D> &a) {
    Fp<D> one_raw = Fp<D>::zero();
    one_raw.v[0] = 1;
    return a * one_raw;
}

// a^e for an exponent given as 32-bit little-endian words (used on host / rarely on device)
template <class D>
MI_HD Fp<D> pow_words(const Fp<D> &a, const uint32_t *e, int nwords) {
    Fp<D> r = Fp<D>::one();
    for (int i = nwords - 1; i >= 0; i--)
        for (int b = 31; b >= 0; b--) {
            r = sqr(r);
            if ((e[i] >> b) & 1) r = r * a;
        }
    return r;
}
template <class D>
MI_HD Fp<D> pow_u64(const Fp<D> &a, uint64_t e) {
    uint32_t w[2] = {(uint32_t)e, (uint32_t)(e >> 32)};
    return pow_words(a, w, 2);
}
template <class D>
MI_NOINL Fp<D> inverse(const Fp<D> &a) {  // Fermat: a^(p-2)
    uint32_t e[D::N];
    for (int i = 0; i < D::N; i++) e[i] = D::MOD[i];
    e[0] -= 2;  // both moduli have low word >= 2 (Fq: ..aaab, Fr: ...0001 -> handle borrow)
    if (D::MOD[0] < 2) {
        // Fr: low word 1 -> 0xffffffff with a borrow into word 1 (word 1 is non-zero)
        e[0] = D::MOD[0] + 0xfffffffeu;
        e[1] = D::MOD[1] - 1;
    }
    return pow_words(a, e, D::N);
}
// a >= b on canonical integers (used for lexicographic sign bits)
template <class D>
MI_HD bool geq_raw(const Fp<D> &a, const Fp<D> &b) {
    for (int i = D::N - 1; i >= 0; i--)
        if (a.v[i] != b.v[i]) return a.v[i] > b.v[i];
    return true;
}

typedef Fp<FqDesc> fq32_t;  // canonical 12 x 32-bit container (wire format conversions only)
typedef Fp<FrDesc> fr_t;

// ---------------------------------------------------------------------------------------------
// Fq: 14 x 29-bit limbs, Montgomery form with R = 2^406, values in [0, 2p)
// ---------------------------------------------------------------------------------------------
struct Fq29 {
    static constexpr int L = 14;
    static constexpr uint32_t M = (1u << 29) - 1;
    static constexpr uint32_t INV = 0x1ffcfffdu;  // -p^-1 mod 2^29
    static constexpr uint32_t P[14] = {0x1fffaaabu, 0x0ff7ffffu, 0x14ffffeeu, 0x17fffd62u, 0x0f6241eau,
                                       0x09507b58u, 0x0afd9cc3u, 0x109e70a2u, 0x1764774bu, 0x121a5d66u,
                                       0x12c6e9edu, 0x12ffcd34u, 0x00111ea3u, 0x0000000du};
    static constexpr uint32_t P2[14] = {0x1fff5556u, 0x1fefffffu, 0x09ffffdcu, 0x0ffffac5u, 0x1ec483d5u,
                                        0x12a0f6b0u, 0x15fb3986u, 0x013ce144u, 0x0ec8ee97u, 0x0434bacdu,
                                        0x058dd3dbu, 0x05ff9a69u, 0x00223d47u, 0x0000001au};
    static constexpr uint32_t ONE[14] = {0x03a9fb84u, 0x0ba00690u, 0x071288f1u, 0x0f59bcc5u, 0x126cb614u,
                                         0x0585bf36u, 0x1b85ac3du, 0x1cf856fau, 0x1891ecbdu, 0x1a7eec05u,
                                         0x155a88f0u, 0x0741ac6du, 0x1317c30fu, 0x00000009u};
    static constexpr uint32_t R2[14] = {0x15bef7aeu, 0x1031cd0eu, 0x02dd93e8u, 0x09226323u, 0x0e6e2cd2u,
                                        0x11684daau, 0x1170e5dbu, 0x088e25b1u, 0x1b366399u, 0x1c536f47u,
                                        0x0d1f9cbcu, 0x0278b67fu, 0x1ea66a2bu, 0x0000000cu};
    // p - 2 as 32-bit words (Fermat inversion exponent)
    static constexpr uint32_t PM2[12] = {0xffffaaa9u, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu,
                                         0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu, 0x64774b84u,
                                         0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
};

struct alignas(8) fq_t {
    static constexpr int L = 14;
    uint32_t v[14];
    MI_HD static fq_t zero() {
        fq_t r;
        MI_UNROLL for (int i = 0; i < L; i++) r.v[i] = 0;
        return r;
    }
    MI_HD static fq_t one() {
        fq_t r;
        MI_UNROLL for (int i = 0; i < L; i++) r.v[i] = Fq29::ONE[i];
        return r;
    }
    // value == 0 mod p (representatives 0 and p)
    MI_HD bool is_zero() const {
        uint32_t z = 0, q = 0;
        MI_UNROLL for (int i = 0; i < L; i++) {
            z |= v[i];
            q |= v[i] ^ Fq29::P[i];
        }
        return z == 0 || q == 0;
    }
    MI_HD bool operator==(const fq_t &o) const;
    MI_HD bool operator!=(const fq_t &o) const { return !(*this == o); }
};

// s - 2p if s >= 2p else s;  s normalised, s < 4p
MI_HD fq_t fq_sub_2p_if_ge(const uint32_t *s) {
    fq_t d;
    int32_t bw = 0;
    MI_UNROLL for (int i = 0; i < 13; i++) {
        int32_t t = (int32_t)s[i] - (int32_t)Fq29::P2[i] + bw;
        d.v[i] = (uint32_t)t & Fq29::M;
        bw = t >> 29;
    }
    int32_t top = (int32_t)s[13] - (int32_t)Fq29::P2[13] + bw;
    d.v[13] = (uint32_t)top;
    if (top < 0) {
        MI_UNROLL for (int i = 0; i < 14; i++) d.v[i] = s[i];
    }
    return d;
}

MI_HD fq_t operator+(const fq_t &a, const fq_t &b) {
    uint32_t s[14];
    uint32_t c = 0;
    MI_UNROLL for (int i = 0; i < 13; i++) {
        uint32_t t = a.v[i] + b.v[i] + c;
        s[i] = t & Fq29::M;
        c = t >> 29;
    }
    s[13] = a.v[13] + b.v[13] + c;
    return fq_sub_2p_if_ge(s);
}

MI_HD fq_t operator-(const fq_t &a, const fq_t &b) {  // a - b + 2p, then reduce below 2p
    uint32_t s[14];
    int32_t c = 0;
    MI_UNROLL for (int i = 0; i < 13; i++) {
        int32_t t = (int32_t)a.v[i] - (int32_t)b.v[i] + (int32_t)Fq29::P2[i] + c;
        s[i] = (uint32_t)t & Fq29::M;
        c = t >> 29;
    }
    s[13] = (uint32_t)((int32_t)a.v[13] - (int32_t)b.v[13] + (int32_t)Fq29::P2[13] + c);
    return fq_sub_2p_if_ge(s);
}

MI_HD fq_t operator-(const fq_t &a) { return fq_t::zero() - a; }
MI_HD fq_t dbl(const fq_t &a) { return a + a; }

// ---- lazy forms: values that only feed multiplications skip the conditional subtraction ----
// REDC(a b) = (a b + m p) / R < a b / R + p, so a product is < 2p whenever a b < p R; with
// R = 2^406 > 2^25 p that holds for operands up to ~2^12 p each.  The column-sum bound of operator*
// and mul_add (<= 42 products per column) needs carry-normalised 29-bit limbs, not values < 2p, so
// an unreduced but normalised operand in [0, 4p) costs nothing.  (The group law keeps every value it
// tests with is_zero or stores reduced to [0, 2p).)
struct Fq29L {
    static constexpr uint32_t P4[14] = {0x1ffeaaacu, 0x1fdfffffu, 0x13ffffb9u, 0x1ffff58au, 0x1d8907aau,
                                        0x0541ed61u, 0x0bf6730du, 0x0279c289u, 0x1d91dd2eu, 0x0869759au,
                                        0x0b1ba7b6u, 0x0bff34d2u, 0x00447a8eu, 0x00000034u};
    static constexpr uint32_t P6[14] = {0x1ffe0002u, 0x1fcfffffu, 0x1dffff96u, 0x0ffff04fu, 0x1c4d8b80u,
                                        0x17e2e412u, 0x01f1ac93u, 0x03b6a3ceu, 0x0c5acbc5u, 0x0c9e3068u,
                                        0x10a97b91u, 0x11fecf3bu, 0x0066b7d5u, 0x0000004eu};
};

// a - b + 2p for b <= 2p: normalised limbs, value in [0, a + 2p) (not reduced)
MI_HD fq_t fq_sub_lazy(const fq_t &a, const fq_t &b) {
    fq_t s;
    int32_t c = 0;
    MI_UNROLL for (int i = 0; i < 13; i++) {
        int32_t t = (int32_t)a.v[i] - (int32_t)b.v[i] + (int32_t)Fq29::P2[i] + c;
        s.v[i] = (uint32_t)t & Fq29::M;
        c = t >> 29;
    }
    s.v[13] = (uint32_t)((int32_t)a.v[13] - (int32_t)b.v[13] + (int32_t)Fq29::P2[13] + c);
    return s;
}

// -y of an affine coordinate y in [0, 2p] as 2p - y (in [0, 2p]); the raw zero stays zero so the
// (0, 0) infinity encoding survives negation
MI_HD fq_t fq_neg_lazy(const fq_t &y) {
    uint32_t z = 0;
    MI_UNROLL for (int i = 0; i < 14; i++) z |= y.v[i];
    const fq_t s = fq_sub_lazy(fq_t::zero(), y);
    fq_t r;
    MI_UNROLL for (int i = 0; i < 14; i++) r.v[i] = z ? s.v[i] : 0u;
    return r;
}

// X3 = R^2 - PPP - 2Q of the XYZZ additions, reduced to [0, 2p): one signed limb pass computes
// R^2 + 6p - PPP - 2Q in [0, 8p) (all three inputs < 2p), then 4p and 2p are conditionally subtracted
// (instead of three add/sub passes with a conditional subtraction each).
MI_HD fq_t fq_x3(const fq_t &r2, const fq_t &ppp, const fq_t &q) {
    uint32_t s[14];
    int32_t c = 0;
    MI_UNROLL for (int i = 0; i < 13; i++) {
        int32_t t = (int32_t)r2.v[i] + (int32_t)Fq29L::P6[i] - (int32_t)ppp.v[i] - 2 * (int32_t)q.v[i] + c;
        s[i] = (uint32_t)t & Fq29::M;
        c = t >> 29;
    }
    s[13] = (uint32_t)((int32_t)r2.v[13] + (int32_t)Fq29L::P6[13] - (int32_t)ppp.v[13] - 2 * (int32_t)q.v[13] + c);
    uint32_t d[14];
    int32_t bw = 0;
    MI_UNROLL for (int i = 0; i < 13; i++) {
        int32_t t = (int32_t)s[i] - (int32_t)Fq29L::P4[i] + bw;
        d[i] = (uint32_t)t & Fq29::M;
        bw = t >> 29;
    }
    const int32_t top = (int32_t)s[13] - (int32_t)Fq29L::P4[13] + bw;
    d[13] = (uint32_t)top;
    if (top < 0) {
        MI_UNROLL for (int i = 0; i < 14; i++) d[i] = s[i];
    }
    return fq_sub_2p_if_ge(d);
}

// canonical representative in [0, p)
MI_HD fq_t fq_canon(const fq_t &a) {
    fq_t d;
    int32_t bw = 0;
    MI_UNROLL for (int i = 0; i < 13; i++) {
        int32_t t = (int32_t)a.v[i] - (int32_t)Fq29::P[i] + bw;
        d.v[i] = (uint32_t)t & Fq29::M;
        bw = t >> 29;
    }
    int32_t top = (int32_t)a.v[13] - (int32_t)Fq29::P[13] + bw;
    d.v[13] = (uint32_t)top;
    return top < 0 ? a : d;
}

MI_HD bool fq_t::operator==(const fq_t &o) const {
    fq_t a = fq_canon(*this), b = fq_canon(o);
    uint32_t x = 0;
    MI_UNROLL for (int i = 0; i < L; i++) x |= a.v[i] ^ b.v[i];
    return x == 0;
}

// Product-scanning Montgomery multiplication, a, b < 2p -> a b R^-1 mod p in [0, 2p).
MI_HD fq_t operator*(const fq_t &a, const fq_t &b) {
    constexpr int L = 14;
    uint32_t m[L];
    fq_t r;
    uint64_t acc = 0;
    MI_UNROLL for (int k = 0; k < L; k++) {
        MI_UNROLL for (int i = 0; i < k; i++) {
            acc += (uint64_t)a.v[i] * b.v[k - i];
            acc += (uint64_t)m[i] * Fq29::P[k - i];
        }
        acc += (uint64_t)a.v[k] * b.v[0];
        m[k] = ((uint32_t)acc * Fq29::INV) & Fq29::M;
        acc += (uint64_t)m[k] * Fq29::P[0];
        acc >>= 29;
    }
    MI_UNROLL for (int k = L; k < 2 * L - 1; k++) {
        MI_UNROLL for (int i = k - L + 1; i < L; i++) {
            acc += (uint64_t)a.v[i] * b.v[k - i];
            acc += (uint64_t)m[i] * Fq29::P[k - i];
        }
        r.v[k - L] = (uint32_t)acc & Fq29::M;
        acc >>= 29;
    }
    r.v[L - 1] = (uint32_t)acc;
    return r;
}
// Squaring: the same product scanning over the symmetric products only -- column k takes
// (2 a_i) a_(k-i) for i < k - i and a_(k/2)^2 -- so the product half costs 105 MADs instead of 196
// (301 instead of 392 in all).  2 a_i < 2^30 for the normalised limbs 0..12 and for a top limb below
// 2^16 (operands < 2^12 p), so each column stays within operator*'s bound (pair products < 2^59, at most
// 7 of them, plus 14 reduction products < 2^58).
MI_HD fq_t sqr(const fq_t &a) {
    constexpr int L = 14;
    uint32_t a2[L];
    MI_UNROLL for (int i = 0; i < L; i++) a2[i] = a.v[i] << 1;
    uint32_t m[L];
    fq_t r;
    uint64_t acc = 0;
    MI_UNROLL for (int k = 0; k < L; k++) {
        MI_UNROLL for (int i = 0; i < k - i; i++) acc += (uint64_t)a2[i] * a.v[k - i];
        if ((k & 1) == 0) acc += (uint64_t)a.v[k >> 1] * a.v[k >> 1];
        MI_UNROLL for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * Fq29::P[k - i];
        m[k] = ((uint32_t)acc * Fq29::INV) & Fq29::M;
        acc += (uint64_t)m[k] * Fq29::P[0];
        acc >>= 29;
    }
    MI_UNROLL for (int k = L; k < 2 * L - 1; k++) {
        MI_UNROLL for (int i = k - L + 1; i < k - i; i++) acc += (uint64_t)a2[i] * a.v[k - i];
        if ((k & 1) == 0) acc += (uint64_t)a.v[k >> 1] * a.v[k >> 1];
        MI_UNROLL for (int i = k - L + 1; i < L; i++) acc += (uint64_t)m[i] * Fq29::P[k - i];
        r.v[k - L] = (uint32_t)acc & Fq29::M;
        acc >>= 29;
    }
    r.v[L - 1] = (uint32_t)acc;
    return r;
}

// a*b + c*d with ONE Montgomery reduction (the group law's "X * Y - Z * W" with c = -Z in lazy
// form): 392 + 196 MADs instead of 2 x 392 plus a subtraction.  Column sums stay below 2^64:
// <= 28 products < 2^58 + 14 reduction products < 2^58 + a carry < 2^35 (42 * 2^58 < 2^63.4).
// Output < (8p^2 + R p) / R < 2p for inputs in [0, 2p) since 8p < R = 2^406.
MI_HD fq_t mul_add(const fq_t &a, const fq_t &b, const fq_t &c, const fq_t &d) {
    constexpr int L = 14;
    uint32_t m[L];
    fq_t r;
    uint64_t acc = 0;
    MI_UNROLL for (int k = 0; k < L; k++) {
        MI_UNROLL for (int i = 0; i < k; i++) {
            acc += (uint64_t)a.v[i] * b.v[k - i];
            acc += (uint64_t)c.v[i] * d.v[k - i];
            acc += (uint64_t)m[i] * Fq29::P[k - i];
        }
        acc += (uint64_t)a.v[k] * b.v[0];
        acc += (uint64_t)c.v[k] * d.v[0];
        m[k] = ((uint32_t)acc * Fq29::INV) & Fq29::M;
        acc += (uint64_t)m[k] * Fq29::P[0];
        acc >>= 29;
    }
    MI_UNROLL for (int k = L; k < 2 * L - 1; k++) {
        MI_UNROLL for (int i = k - L + 1; i < L; i++) {
            acc += (uint64_t)a.v[i] * b.v[k - i];
            acc += (uint64_t)c.v[i] * d.v[k - i];
            acc += (uint64_t)m[i] * Fq29::P[k - i];
        }
        r.v[k - L] = (uint32_t)acc & Fq29::M;
        acc >>= 29;
    }
    r.v[L - 1] = (uint32_t)acc;
    return r;
}

// canonical 12 x 32-bit integer (< p) -> Montgomery
MI_HD fq_t fq_from_raw(const fq32_t &raw) {
    fq_t t;
    MI_UNROLL for (int i = 0; i < 14; i++) {
        const int bit = 29 * i, w = bit >> 5, s = bit & 31;
        uint64_t x = raw.v[w];
        if (w + 1 < 12) x |= (uint64_t)raw.v[w + 1] << 32;
        t.v[i] = (uint32_t)(x >> s) & Fq29::M;
    }
    fq_t r2;
    MI_UNROLL for (int i = 0; i < 14; i++) r2.v[i] = Fq29::R2[i];
    return t * r2;
}
// Montgomery -> canonical 12 x 32-bit integer (< p)
MI_HD fq32_t fq_to_raw(const fq_t &a) {
    fq_t one = fq_t::zero();
    one.v[0] = 1;
    fq_t c = fq_canon(a * one);
    fq32_t r = fq32_t::zero();
    MI_UNROLL for (int i = 0; i < 14; i++) {
        const int bit = 29 * i, w = bit >> 5, s = bit & 31;
        r.v[w] |= c.v[i] << s;
        if (s > 3 && w + 1 < 12) r.v[w + 1] |= c.v[i] >> (32 - s);
    }
    return r;
}
MI_HD fq_t fq_small(uint32_t v) {
    fq32_t r = fq32_t::zero();
    r.v[0] = v;
    return fq_from_raw(r);
}
// Fermat inversion a^(p-2).  *_inl versions are for device kernels (no device-side calls: large
// noinline functions with big by-value structs miscompile / overflow the stack on gfx950).
MI_HD fq_t inverse_inl(const fq_t &a) {
    fq_t r = fq_t::one();
#pragma unroll 1
    for (int i = 11; i >= 0; i--)
#pragma unroll 1
        for (int b = 31; b >= 0; b--) {
            r = sqr(r);
            if ((Fq29::PM2[i] >> b) & 1) r = r * a;
        }
    return r;
}
MI_NOINL fq_t inverse(const fq_t &a) { return inverse_inl(a); }

// ---------------------------------------------------------------------------------------------
// Fq2 = Fq[u]/(u^2 + 1)  (G2 coordinates)
// ---------------------------------------------------------------------------------------------
struct alignas(16) fq2_t {
    fq_t c0, c1;
    MI_HD static fq2_t zero() { return {fq_t::zero(), fq_t::zero()}; }
    MI_HD static fq2_t one() { return {fq_t::one(), fq_t::zero()}; }
    MI_HD bool is_zero() const { return c0.is_zero() && c1.is_zero(); }
    MI_HD bool operator==(const fq2_t &o) const { return c0 == o.c0 && c1 == o.c1; }
    MI_HD bool operator!=(const fq2_t &o) const { return !(*this == o); }
};
MI_HD fq2_t operator+(const fq2_t &a, const fq2_t &b) { return {a.c0 + b.c0, a.c1 + b.c1}; }
MI_HD fq2_t operator-(const fq2_t &a, const fq2_t &b) { return {a.c0 - b.c0, a.c1 - b.c1}; }
MI_HD fq2_t operator-(const fq2_t &a) { return {-a.c0, -a.c1}; }
MI_HD fq2_t dbl(const fq2_t &a) { return a + a; }
MI_HD fq2_t operator*(const fq2_t &a, const fq2_t &b) {  // Karatsuba, 3 Fq mults
    fq_t v0 = a.c0 * b.c0, v1 = a.c1 * b.c1;
    fq_t t = (a.c0 + a.c1) * (b.c0 + b.c1);
    return {v0 - v1, t - v0 - v1};
}
MI_HD fq2_t mul_add(const fq2_t &a, const fq2_t &b, const fq2_t &c, const fq2_t &d) { return a * b + c * d; }
MI_HD fq2_t sqr(const fq2_t &a) {  // (a0 + a1)(a0 - a1), 2 a0 a1: 2 Fq mults
    fq_t t = a.c0 * a.c1;
    return {(a.c0 + a.c1) * (a.c0 - a.c1), t + t};
}
MI_HD fq2_t inverse_inl(const fq2_t &a) {
    fq_t n = inverse_inl(sqr(a.c0) + sqr(a.c1));
    return {a.c0 * n, -(a.c1 * n)};
}
MI_NOINL fq2_t inverse(const fq2_t &a) { return inverse_inl(a); }

}  // namespace mi
