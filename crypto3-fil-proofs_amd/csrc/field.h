// field.h -- BLS12-381 base field Fq (381-bit) and scalar field Fr (255-bit) in Montgomery form.
//
// Restates crypto3's multiprecision Montgomery backend ([NOT IN TREE]: libs/crypto/multiprecision,
// used via algebra::curves::bls12<381>, core/crypto/scheme_params.hpp:39-43) for CDNA4:
//   * Fq (the MSM hot loop) uses 13 balanced signed limbs of 30 bits, Montgomery radix R = 2^390,
//     product-scanning (FIPS) Montgomery multiplication: a column holds <= 26 products of magnitude
//     <= 2^58, so every limb product is ONE v_mad_i64_i32 accumulating into a signed 64-bit register
//     pair and carries move once per column (338 MADs; 84 G Fq-mul/s on MI355X against 79 for the
//     rounds 1-4 form over 14 x 29-bit unsigned limbs and 38 for 32-bit CIOS, microbench/fieldmul.hip).
//     Values are any representative (no range reduction); see "Fq" below.
//   * Fr (NTT, scalars) uses 8 limbs of 32 bits with "no-carry" CIOS (top limb < 2^31 - 1); its
//     memory image is the canonical 32-byte little-endian encoding.
//   * everything is fully unrolled so elements live in VGPRs (Fq = 13, Fr = 8 registers).
// The same code compiles for the host (final window combination, proof assembly).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MI_HD __host__ __device__ __forceinline__
#define MI_UNROLL _Pragma("unroll")
// group-law level functions are compiled once and called (keeps kernels and build times small)
#define MI_NOINL __host__ __device__ __attribute__((noinline)) inline

namespace mi {

// MI_FQ_CHECK (a debug build, `make fqcheck`; off in release): the device group law counts violations of the Fq
// magnitude invariant instead of trusting the comments -- [0] a normalised value with |top limb| > 2^24 (|V| beyond
// ~9.8 p: fq_norm's host-only magnitude control would have been needed), [1] fq_is_zero with |round(V / p)| > 3 (the
// group law's sums are argued to stay below 3 p).  Counters, not asserts: a device trap would fault the GPU.  Each
// translation unit has its own counters and registers their host shadow at load (mi_fq_check_read sums them).
// Round 6, the MSM / window-table / prove parity tests under the debug build (profiles/r06/fq_check_debug_build.log):
// the top-limb bound held in every unit (largest |top limb| 11 x 2^20 of the 16 x 2^20 allowed); the MSM units never
// zero-tested |k| > 3; prover.hip's key-table doubling chains (window / split tables, key generation) did so 1,694
// times with |k| = 4, which fq_is_zero's reduction loop handles -- so |k| <= 3 is the MSM group law's property, not
// a library-wide one, and the loop is what makes the zero test exact everywhere.
#ifdef MI_FQ_CHECK
// [0], [1] the two counts above, [2] the largest |round(V / p)| a zero test saw, [3] the largest |top limb| >> 20
__device__ static unsigned int g_fq_check[4];
void fq_check_register(const void *symbol, const char *unit);
struct FqCheckRegistrar {
    FqCheckRegistrar() { fq_check_register((const void *)&g_fq_check, __BASE_FILE__); }
};
static FqCheckRegistrar g_fq_check_registrar;
#define MI_FQ_CHECK_HIT(i) atomicAdd(&g_fq_check[i], 1u)
#define MI_FQ_CHECK_MAX(i, v) atomicMax(&g_fq_check[i], (unsigned int)(v))
#endif

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
// Fq: 13 x 30-bit BALANCED SIGNED limbs, Montgomery form with R = 2^390
// ---------------------------------------------------------------------------------------------
// A value is V = sum_i v_i 2^(30 i) with limbs 0..11 normalised to [-2^29, 2^29] and a small signed top
// limb; V is any representative of its residue (no range reduction in add / sub / neg), |V| < 2^388.
// Why balanced 30-bit limbs (round 5, microbench/fieldmul.hip): a limb product is at most 2^58 in
// magnitude, so a product-scanning column of 13 a*b + 13 m*p products stays inside a signed 64-bit
// accumulator (26 * 2^58 = 2^62.7) and every limb product is ONE v_mad_i64_i32: 338 per Montgomery
// product instead of the 392 v_mad_u64_u32 of 14 x 29-bit unsigned limbs (84.3 vs 79.0 G Fq-mul/s on
// MI355X, same box).  Unsigned 30-bit limbs would overflow the column (26 * 2^60).  Signed limbs also make
// negation free (limb-wise) and let add / sub skip the conditional subtraction of 2p: they only carry-
// normalise.  The Montgomery output satisfies |out| <= |a b| / R + p / 2 (m has balanced digits too), so
// products pull every magnitude back below ~0.52 p for operands below 3 p, the group law's range.
// Equality and is_zero work modulo p for any representative (quotient estimate from the top limb, then an
// exact limb check), so no caller depends on a reduced range.
struct Fq30 {
    static constexpr int L = 13;
    static constexpr uint32_t M = (1u << 30) - 1;
    static constexpr uint32_t INV = 0x3ffcfffdu;  // -p^-1 mod 2^30
    static constexpr int32_t P[13] = {-21845,     -402915328, 356515836, -352321620, -252304353, 55215067, 288093811,
                                      316751073,  -321428361, 517541167, -375082566, -91332614,  1704210};
    static constexpr int32_t ONE[13] = {13762350,   433586176, -192935228, -301937177, 37952645, -425753694, -36732706,
                                        162803105,  -437337492, 366579475, 78814996,   -442511456, 89578};
    static constexpr int32_t R2[13] = {84936463,   -82245875, 20063291,   -375672600, -184045713, -75371400, -508475920,
                                       172522421,  -150322876, 98350284,  415856896,  -132992156, 1010031};
    // round(2^51 / (p / 2^360)) < 2^31: quotient estimate k = round(V / p) from the top limb alone (exact for V = k p)
    static constexpr int32_t QINV = 1321315992;
    // p - 2 as 32-bit words (Fermat inversion exponent)
    static constexpr uint32_t PM2[12] = {0xffffaaa9u, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu,
                                         0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu, 0x64774b84u,
                                         0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
};

MI_HD int32_t fq_sext30(uint32_t x) { return ((int32_t)(x << 2)) >> 2; }

// The operands of the limb products as plain 32-bit registers.  Inside the inlined group law LLVM widens limbs that
// live across loop iterations to 64-bit values and then no longer sees that (int64) a_i * b_j is a product of two
// sign-extended 32-bit values: it emits a 64 x 64 multiply (v_mad_u64_u32 + 2 v_mul_lo_u32 + v_add3) instead of one
// v_mad_i64_i32.  An empty asm on each 32-bit limb (device only) pins the value at 32 bits.
MI_HD void fq_pin(int32_t *x, const int32_t *a) {
#pragma unroll
    for (int i = 0; i < 13; i++) {
        x[i] = a[i];
#if defined(__HIP_DEVICE_COMPILE__)
        asm("" : "+v"(x[i]));
#endif
    }
}

struct fq_t;
MI_HD bool fq_is_zero(const fq_t &a);

struct alignas(8) fq_t {
    static constexpr int L = 13;
    int32_t v[13];
    MI_HD static fq_t zero() {
        fq_t r;
        MI_UNROLL for (int i = 0; i < L; i++) r.v[i] = 0;
        return r;
    }
    MI_HD static fq_t one() {
        fq_t r;
        MI_UNROLL for (int i = 0; i < L; i++) r.v[i] = Fq30::ONE[i];
        return r;
    }
    // value == 0 mod p, for any representative
    MI_HD bool is_zero() const { return fq_is_zero(*this); }
    // all limbs zero: the exact test for values that are zero only as the raw 0 (products, stored coordinates)
    MI_HD bool is_raw_zero() const {
        uint32_t z = 0;
        MI_UNROLL for (int i = 0; i < L; i++) z |= (uint32_t)v[i];
        return z == 0;
    }
    MI_HD bool operator==(const fq_t &o) const;
    MI_HD bool operator!=(const fq_t &o) const { return !(*this == o); }
};

// round(V / p) from the top limb (|V| < 2^388): the other limbs move V / p by < 2^-21, so the estimate is
// exact whenever V is a multiple of p and within 1 of V / p otherwise
MI_HD int32_t fq_quot(const fq_t &a) { return (int32_t)(((int64_t)a.v[12] * Fq30::QINV + (1ll << 50)) >> 51); }

// V - k p, carry-normalised (limbs 0..11 in [-2^29, 2^29))
MI_HD fq_t fq_sub_kp(const fq_t &a, int32_t k) {
    fq_t r;
    int64_t c = 0;
    MI_UNROLL for (int i = 0; i < 12; i++) {
        const int64_t t = (int64_t)a.v[i] - (int64_t)k * Fq30::P[i] + c;
        r.v[i] = fq_sext30((uint32_t)t);
        c = (t + (1 << 29)) >> 30;
    }
    r.v[12] = (int32_t)((int64_t)a.v[12] - (int64_t)k * Fq30::P[12] + c);
    return r;
}

// V - j p for |j| <= 3 in 32-bit arithmetic (|v_i - j p_i + c| < 2^29 + 1.56e9 + 2 < 2^31), carry-normalised
MI_HD fq_t fq_sub_small(const fq_t &a, int32_t j) {
    fq_t r;
    int32_t c = 0;
    MI_UNROLL for (int i = 0; i < 12; i++) {
        const int32_t t = a.v[i] - j * Fq30::P[i] + c;
        r.v[i] = fq_sext30((uint32_t)t);
        c = ((t >> 29) + 1) >> 1;  // round(t / 2^30) = (t - r_i) / 2^30 without forming t - r_i (up to 2^31)
    }
    r.v[12] = a.v[12] - j * Fq30::P[12] + c;
    return r;
}
// a == k p exactly, |k| <= 3: the balanced digits of k p are formed on the fly (32-bit) and compared limb by limb.
// Exact because no canonical digit of k p (|k| <= 3) is -2^29, so k p has one representation with digits in
// [-2^29, 2^29] (checked when the constants were derived) and any normalised a equal to it has those digits.
MI_HD bool fq_is_kp(const fq_t &a, int32_t k) {
    int32_t c = 0;
    uint32_t diff = 0;
    MI_UNROLL for (int i = 0; i < 12; i++) {
        const int32_t t = k * Fq30::P[i] + c;
        const int32_t d = fq_sext30((uint32_t)t);
        c = (t - d) >> 30;
        diff |= (uint32_t)(a.v[i] - d);
    }
    diff |= (uint32_t)(a.v[12] - (k * Fq30::P[12] + c));
    return diff == 0;
}

// V == 0 mod p: with k = round(V / p), V is a multiple of p iff V = k p, which first needs the low limb to
// match (one 32-bit check, the hot path); only then (never, for random data) are all limbs compared, in 32-bit
// register-light steps (an inlined 64-bit V - k p here cost the accumulation kernel 50 registers)
MI_HD bool fq_is_zero(const fq_t &a) {
    int32_t k = fq_quot(a);
#if defined(MI_FQ_CHECK) && defined(__HIP_DEVICE_COMPILE__)
    if (k > 3 || k < -3) {
        MI_FQ_CHECK_HIT(1);
        MI_FQ_CHECK_MAX(2, k < 0 ? -k : k);
    }
#endif
    if ((((uint32_t)a.v[0] - (uint32_t)k * (uint32_t)Fq30::P[0]) & Fq30::M) != 0) return false;
    fq_t x = a;
    while (k > 3) {  // only far-out representatives (never in the group law, whose values stay below 3 p)
        x = fq_sub_small(x, 3);
        k -= 3;
    }
    while (k < -3) {
        x = fq_sub_small(x, -3);
        k += 3;
    }
    return fq_is_kp(x, k);
}

// carry-normalise limb sums t_i of two normalised operands (|t_i| <= 2^30, so t_i + carry + 2^29 < 2^31):
// limbs 0..11 into [-2^29, 2^29), the carry into the top
MI_HD fq_t fq_norm(const int32_t *t) {
    fq_t r;
    int32_t c = 0;
    MI_UNROLL for (int i = 0; i < 12; i++) {
        const int32_t x = t[i] + c;
        c = (x + (1 << 29)) >> 30;
        r.v[i] = x - (int32_t)((uint32_t)c << 30);
    }
    r.v[12] = t[12] + c;
    // Magnitude control: products come out below ~0.7 p whatever their inputs, but a value rebuilt from sums alone
    // (the Miller loop's affine x3 = lambda^2 - 2 x, iterated) would double each time.  Past |V| ~ 2^384 (top limb
    // 2^24, ~9.8 p) subtract round(V / p) p.  The group law's sums stay below 3 p, so the MSM kernels never take
    // this branch.
#if !defined(__HIP_DEVICE_COMPILE__)
    const int32_t top = r.v[12] < 0 ? -r.v[12] : r.v[12];
    if (__builtin_expect(top > (1 << 24), 0)) r = fq_sub_kp(r, fq_quot(r));
#elif defined(MI_FQ_CHECK)
    if (r.v[12] > (1 << 24) || r.v[12] < -(1 << 24)) MI_FQ_CHECK_HIT(0);
    MI_FQ_CHECK_MAX(3, (r.v[12] < 0 ? -r.v[12] : r.v[12]) >> 20);
#endif
    return r;
}

MI_HD fq_t operator+(const fq_t &a, const fq_t &b) {
    int32_t t[13];
    MI_UNROLL for (int i = 0; i < 13; i++) t[i] = a.v[i] + b.v[i];
    return fq_norm(t);
}
MI_HD fq_t operator-(const fq_t &a, const fq_t &b) {
    int32_t t[13];
    MI_UNROLL for (int i = 0; i < 13; i++) t[i] = a.v[i] - b.v[i];
    return fq_norm(t);
}
MI_HD fq_t operator-(const fq_t &a) {  // limb-wise: |-v_i| <= 2^29 stays normalised, and -0 = 0
    fq_t r;
    MI_UNROLL for (int i = 0; i < 13; i++) r.v[i] = -a.v[i];
    return r;
}
MI_HD fq_t dbl(const fq_t &a) { return a + a; }

// The group law's former lazy forms (values feeding only multiplications skipped the conditional
// subtraction of the unsigned representation): with signed limbs every add / sub is already "lazy".
MI_HD fq_t fq_sub_lazy(const fq_t &a, const fq_t &b) { return a - b; }
MI_HD fq_t fq_neg_lazy(const fq_t &y) { return -y; }
// X3 = R^2 - PPP - 2Q (three two-operand passes: a three-operand limb sum plus the rounding bias of fq_norm
// could reach 2^31)
MI_HD fq_t fq_x3(const fq_t &r2, const fq_t &ppp, const fq_t &q) { return (r2 - ppp) - dbl(q); }

// sign of the value (-1, 0, 1): the sign of the most significant non-zero limb
MI_HD int fq_sign(const fq_t &a) {
    int s = 0;
    MI_UNROLL for (int i = 0; i < 13; i++) s = a.v[i] > 0 ? 1 : (a.v[i] < 0 ? -1 : s);
    return s;
}
// canonical representative in [0, p), normalised limbs (cold paths: encodings, equality of host values)
MI_HD fq_t fq_canon(const fq_t &a) {
    fq_t d = fq_sub_kp(a, fq_quot(a));  // |d| < p
    if (fq_sign(d) < 0) d = fq_sub_kp(d, -1);
    const fq_t e = fq_sub_kp(d, 1);
    return fq_sign(e) >= 0 ? e : d;
}

MI_HD bool fq_t::operator==(const fq_t &o) const { return fq_is_zero(*this - o); }

// Product-scanning Montgomery multiplication: a b R^-1 mod p, |out| <= |a b| / R + p / 2.
// Column k <= 12 holds <= 13 a*b and 13 m*p products (|.| <= 2^58) plus a carry: < 2^62.71.
MI_HD fq_t operator*(const fq_t &a_, const fq_t &b_) {
    constexpr int L = 13;
    struct {
        int32_t v[13];
    } a, b;
    fq_pin(a.v, a_.v);
    fq_pin(b.v, b_.v);
    int32_t m[L];
    fq_t r;
    int64_t acc = 0;
    MI_UNROLL for (int k = 0; k < L; k++) {
        MI_UNROLL for (int i = 0; i < k; i++) {
            acc += (int64_t)a.v[i] * b.v[k - i];
            acc += (int64_t)m[i] * Fq30::P[k - i];
        }
        acc += (int64_t)a.v[k] * b.v[0];
        m[k] = fq_sext30((uint32_t)acc * Fq30::INV);
        acc += (int64_t)m[k] * Fq30::P[0];
        acc >>= 30;  // exact: the low 30 bits are zero
    }
    MI_UNROLL for (int k = L; k < 2 * L - 1; k++) {
        MI_UNROLL for (int i = k - L + 1; i < L; i++) {
            acc += (int64_t)a.v[i] * b.v[k - i];
            acc += (int64_t)m[i] * Fq30::P[k - i];
        }
        r.v[k - L] = fq_sext30((uint32_t)acc);
        acc = (acc + (1 << 29)) >> 30;  // == (acc - sext30(acc)) >> 30
    }
    r.v[L - 1] = (int32_t)acc;
    return r;
}
// Squaring over the symmetric products: column k takes (2 a_i) a_(k-i) for i < k - i (|.| <= 2^59, at most
// 6 of them) and a_(k/2)^2, so the product half costs 91 MADs instead of 169 (260 in all); column bound
// 6 * 2^59 + 14 * 2^58 = 26 * 2^58.
MI_HD fq_t sqr(const fq_t &a_) {
    constexpr int L = 13;
    struct {
        int32_t v[13];
    } a;
    fq_pin(a.v, a_.v);
    int32_t a2[L];
    MI_UNROLL for (int i = 0; i < L; i++) a2[i] = a.v[i] * 2;
    int32_t m[L];
    fq_t r;
    int64_t acc = 0;
    MI_UNROLL for (int k = 0; k < L; k++) {
        MI_UNROLL for (int i = 0; i < k - i; i++) acc += (int64_t)a2[i] * a.v[k - i];
        if ((k & 1) == 0) acc += (int64_t)a.v[k >> 1] * a.v[k >> 1];
        MI_UNROLL for (int i = 0; i < k; i++) acc += (int64_t)m[i] * Fq30::P[k - i];
        m[k] = fq_sext30((uint32_t)acc * Fq30::INV);
        acc += (int64_t)m[k] * Fq30::P[0];
        acc >>= 30;
    }
    MI_UNROLL for (int k = L; k < 2 * L - 1; k++) {
        MI_UNROLL for (int i = k - L + 1; i < k - i; i++) acc += (int64_t)a2[i] * a.v[k - i];
        if ((k & 1) == 0) acc += (int64_t)a.v[k >> 1] * a.v[k >> 1];
        MI_UNROLL for (int i = k - L + 1; i < L; i++) acc += (int64_t)m[i] * Fq30::P[k - i];
        r.v[k - L] = fq_sext30((uint32_t)acc);
        acc = (acc + (1 << 29)) >> 30;
    }
    r.v[L - 1] = (int32_t)acc;
    return r;
}

// a*b + c*d with ONE Montgomery reduction (the group law's Y3 and the G2 lane-pair product): 507 MADs
// instead of 2 x 338.  A column can hold 3 x 13 products, more than the accumulator takes, so in columns
// 10..14 (the only ones with more than 31 products of magnitude 2^58; p_0 and p_12 are small) the a*b and
// m*p part is split into its high part (kept aside) and its low 30 bits before the c*d products go in.
// |out| <= (|a b| + |c d|) / R + p / 2.
MI_HD fq_t mul_add(const fq_t &a_, const fq_t &b_, const fq_t &c_, const fq_t &d_) {
    constexpr int L = 13;
    struct {
        int32_t v[13];
    } a, b, c, d;
    fq_pin(a.v, a_.v);
    fq_pin(b.v, b_.v);
    fq_pin(c.v, c_.v);
    fq_pin(d.v, d_.v);
    int32_t m[L];
    fq_t r;
    int64_t acc = 0;
    MI_UNROLL for (int k = 0; k < L; k++) {
        MI_UNROLL for (int i = 0; i < k; i++) {
            acc += (int64_t)a.v[i] * b.v[k - i];
            acc += (int64_t)m[i] * Fq30::P[k - i];
        }
        acc += (int64_t)a.v[k] * b.v[0];
        int64_t hi = 0;
        if (k >= 10) {
            hi = acc >> 30;
            acc &= Fq30::M;
        }
        MI_UNROLL for (int i = 0; i <= k; i++) acc += (int64_t)c.v[i] * d.v[k - i];
        m[k] = fq_sext30((uint32_t)acc * Fq30::INV);
        acc += (int64_t)m[k] * Fq30::P[0];
        acc = (acc >> 30) + hi;
    }
    MI_UNROLL for (int k = L; k < 2 * L - 1; k++) {
        MI_UNROLL for (int i = k - L + 1; i < L; i++) {
            acc += (int64_t)a.v[i] * b.v[k - i];
            acc += (int64_t)m[i] * Fq30::P[k - i];
        }
        int64_t hi = 0;
        if (k <= 14) {
            hi = acc >> 30;
            acc &= Fq30::M;
        }
        MI_UNROLL for (int i = k - L + 1; i < L; i++) acc += (int64_t)c.v[i] * d.v[k - i];
        r.v[k - L] = fq_sext30((uint32_t)acc);
        acc = ((acc + (1 << 29)) >> 30) + hi;
    }
    r.v[L - 1] = (int32_t)acc;
    return r;
}

// canonical 12 x 32-bit integer (< p) -> Montgomery
MI_HD fq_t fq_from_raw(const fq32_t &raw) {
    int32_t t[13];
    MI_UNROLL for (int i = 0; i < 13; i++) {
        const int bit = 30 * i, w = bit >> 5, s = bit & 31;
        uint64_t x = raw.v[w];
        if (w + 1 < 12) x |= (uint64_t)raw.v[w + 1] << 32;
        t[i] = (int32_t)((uint32_t)(x >> s) & Fq30::M);  // unsigned 30-bit digits, normalised below
    }
    fq_t r2;
    MI_UNROLL for (int i = 0; i < 13; i++) r2.v[i] = Fq30::R2[i];
    return fq_norm(t) * r2;
}
// Montgomery -> canonical 12 x 32-bit integer (< p)
MI_HD fq32_t fq_to_raw(const fq_t &a) {
    fq_t one = fq_t::zero();
    one.v[0] = 1;
    const fq_t c = fq_canon(a * one);
    uint32_t u[13];  // unsigned 30-bit digits of the canonical value
    int32_t cy = 0;
    MI_UNROLL for (int i = 0; i < 13; i++) {
        const int32_t x = c.v[i] + cy;
        u[i] = (uint32_t)x & Fq30::M;
        cy = x >> 30;  // floor
    }
    fq32_t r = fq32_t::zero();
    MI_UNROLL for (int i = 0; i < 13; i++) {
        const int bit = 30 * i, w = bit >> 5, s = bit & 31;
        r.v[w] |= u[i] << s;
        if (s > 2 && w + 1 < 12) r.v[w + 1] |= u[i] >> (32 - s);
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
            if ((Fq30::PM2[i] >> b) & 1) r = r * a;
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
