// field.h -- BLS12-381 base field Fq (381-bit) and scalar field Fr (255-bit) in Montgomery form.
//
// Restates crypto3's multiprecision Montgomery backend ([NOT IN TREE]: libs/crypto/multiprecision,
// used via algebra::curves::bls12<381>, core/crypto/scheme_params.hpp:39-43) for CDNA4:
//   * limbs are 32-bit so every limb product is one v_mad_u64_u32 (32x32+64 -> 64) -- CDNA has no
//     64x64->128 multiplier; the memory image is identical to 64-bit little-endian limbs,
//   * "no-carry" CIOS: both moduli have a top 32-bit limb < 2^31 - 1, so the CIOS inner loops for
//     the product and the reduction merge and the (N+1)th/(N+2)th words disappear,
//   * everything is fully unrolled so elements live in VGPRs (Fq = 12, Fr = 8 registers).
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
    static constexpr uint32_t R1[8] = {0xfffffffeu, 0x00000001u, 0x00034802u, 0x5884b7fau,
                                       0xecbc4ff5u, 0x998c4fefu, 0xacc5056fu, 0x1824b159u};
    static constexpr uint32_t R2[8] = {0xf3f29c6du, 0xc999e990u, 0x87925c23u, 0x2b6cedcbu,
                                       0x7254398fu, 0x05d31496u, 0x9f59ff11u, 0x0748d9d9u};
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

typedef Fp<FqDesc> fq_t;
typedef Fp<FrDesc> fr_t;

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
MI_NOINL fq2_t operator*(const fq2_t &a, const fq2_t &b) {  // Karatsuba, 3 Fq mults
    fq_t v0 = a.c0 * b.c0, v1 = a.c1 * b.c1;
    fq_t t = (a.c0 + a.c1) * (b.c0 + b.c1);
    return {v0 - v1, t - v0 - v1};
}
MI_NOINL fq2_t sqr(const fq2_t &a) {  // (a0 + a1)(a0 - a1), 2 a0 a1: 2 Fq mults
    fq_t t = a.c0 * a.c1;
    return {(a.c0 + a.c1) * (a.c0 - a.c1), t + t};
}
MI_NOINL fq2_t inverse(const fq2_t &a) {
    fq_t n = inverse(sqr(a.c0) + sqr(a.c1));
    return {a.c0 * n, -(a.c1 * n)};
}
MI_HD fq2_t to_mont(const fq2_t &a) { return {to_mont(a.c0), to_mont(a.c1)}; }
MI_HD fq2_t from_mont(const fq2_t &a) { return {from_mont(a.c0), from_mont(a.c1)}; }

}  // namespace mi
