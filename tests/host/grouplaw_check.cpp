// grouplaw_check.cpp -- TEST INFRASTRUCTURE: the device group law (csrc/field.h, csrc/curve.h) compiled
// for the host, checked against the CPU oracle (oracle/, linked) under ASan/UBSan.
//
// The Fq arithmetic the MSM kernels inline works on balanced signed 30-bit limbs with no range reduction
// (field.h "Fq").  This program runs exactly that code on the host over sequences that hit every branch
// of the group law -- distinct points with random signs, P + P (doubling), P + (-P) (infinity), infinity
// operands (the raw (0, 0) encoding), other representatives v + k p of every finite coordinate -- and compares
// each result with the
// oracle's affine group law.  It also checks every field operation against plain integers mod p (an
// independent reference over 32-bit words with reduced additions only), on random values and on limb
// patterns at the column-sum bound (every low limb +-2^29).
// Build/run: tests/test_cpu_grouplaw.py (hipcc host-only, ASan + UBSan, host code only).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "curve.h"
#include "glv.h"
#include "hostfield.h"
#include "oracle.h"
#include "subgroup_vectors.h"

using namespace mi;

static std::mt19937_64 rng(12345);
static int failures = 0;
#define CHECK(cond, ...)                        \
    do {                                        \
        if (!(cond)) {                          \
            std::printf("FAIL %s:%d ", __FILE__, __LINE__); \
            std::printf(__VA_ARGS__);           \
            std::printf("\n");                  \
            failures++;                         \
        }                                       \
    } while (0)

static fq_t fq_from_be(const uint8_t *p) {
    fq32_t raw;
    for (int i = 0; i < 12; i++) {
        const uint8_t *q = p + 4 * (11 - i);
        raw.v[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
    }
    return fq_from_raw(raw);
}
static void fq_to_be(const fq_t &a, uint8_t *p) {
    fq32_t raw = fq_to_raw(a);
    for (int i = 0; i < 12; i++) {
        uint32_t w = raw.v[i];
        uint8_t *q = p + 4 * (11 - i);
        q[0] = w >> 24, q[1] = w >> 16, q[2] = w >> 8, q[3] = w;
    }
}
// another representative of the same residue: v + k p for a random k in [-2, 2] (limbs stay normalised)
static fq_t alt_rep(const fq_t &a) { return fq_sub_kp(fq_canon(a), (int32_t)(rng() % 5) - 2); }
static fq_t rand_fq() {  // random residue, random representative in (-2p, 3p)
    uint8_t b[48];
    for (int i = 0; i < 48; i++) b[i] = (uint8_t)rng();
    b[0] &= 0x0f;  // < 2^380 < p
    fq_t a = fq_from_be(b);
    return (rng() & 1) ? alt_rep(a) : fq_canon(a);
}

// ---- an independent reference for the field checks: values mod p over fq32_t (12 x 32-bit, reduced
// additions only, no Montgomery code), so the signed-limb forms are checked against plain integers ----
static fq32_t ref_add(const fq32_t &a, const fq32_t &b) { return a + b; }  // Fp<FqDesc>: reduced a + b
static fq32_t ref_sub(const fq32_t &a, const fq32_t &b) { return a - b; }
static fq32_t ref_small(uint32_t v) {
    fq32_t r = fq32_t::zero();
    r.v[0] = v;
    return reduce_once(r);
}
// value of a limb vector mod p: Horner over the signed limbs, base 2^30 by doublings
static fq32_t ref_val(const fq_t &a) {
    fq32_t acc = fq32_t::zero();
    for (int i = 12; i >= 0; i--) {
        for (int j = 0; j < 30; j++) acc = ref_add(acc, acc);
        const int32_t v = a.v[i];
        const uint32_t mag = v < 0 ? (uint32_t)(-(int64_t)v) : (uint32_t)v;
        // |v| may exceed p's low word range only as an integer < 2^31, so add it in two halves
        fq32_t m = ref_add(ref_small(mag >> 16), fq32_t::zero());
        for (int j = 0; j < 16; j++) m = ref_add(m, m);
        m = ref_add(m, ref_small(mag & 0xffff));
        acc = v < 0 ? ref_sub(acc, m) : ref_add(acc, m);
    }
    return acc;
}
static fq32_t ref_mul(const fq32_t &a, const fq32_t &b) {  // double-and-add over b's bits
    fq32_t acc = fq32_t::zero();
    for (int i = 11; i >= 0; i--)
        for (int j = 31; j >= 0; j--) {
            acc = ref_add(acc, acc);
            if ((b.v[i] >> j) & 1) acc = ref_add(acc, a);
        }
    return acc;
}
static fq32_t ref_rinv() {  // 2^-390 mod p by 390 halvings of 1
    static const fq32_t P = fq32_t::modulus_raw();
    fq32_t x = ref_small(1);
    for (int k = 0; k < 390; k++) {
        if (x.v[0] & 1) {  // (x + p) / 2 over 13 words
            uint64_t c = 0;
            uint32_t w[13];
            for (int i = 0; i < 12; i++) {
                c += (uint64_t)x.v[i] + P.v[i];
                w[i] = (uint32_t)c;
                c >>= 32;
            }
            w[12] = (uint32_t)c;
            for (int i = 0; i < 12; i++) x.v[i] = (w[i] >> 1) | (w[i + 1] << 31);
        } else {
            for (int i = 0; i < 12; i++) x.v[i] = (x.v[i] >> 1) | (i < 11 ? x.v[i + 1] << 31 : 0);
        }
    }
    return x;
}
static bool ref_eq(const fq32_t &a, const fq32_t &b) { return std::memcmp(a.v, b.v, sizeof a.v) == 0; }
static bool normalised(const fq_t &a) {
    for (int i = 0; i < 12; i++)
        if (a.v[i] < -(1 << 29) || a.v[i] > (1 << 29)) return false;
    return a.v[12] >= -(1 << 29) && a.v[12] <= (1 << 29);
}
// limb patterns at the column-sum bound: every low limb +-2^29 (or random extremes), moderate top limb
static fq_t extreme_fq(int kind) {
    fq_t a;
    for (int i = 0; i < 12; i++) {
        const int sgn = kind == 0 ? 1 : kind == 1 ? -1 : ((rng() & 1) ? 1 : -1);
        a.v[i] = sgn * (1 << 29);
    }
    a.v[12] = (int32_t)(rng() % 4000001) - 2000000;  // |V| up to ~1.2 p
    return a;
}

static void g1_to_bytes(const g1_affine_t &a, uint8_t out[96]) {
    if (a.is_inf()) {
        std::memset(out, 0, 96);
        out[0] = 0x40;
        return;
    }
    fq_to_be(a.x, out);
    fq_to_be(a.y, out + 48);
}
static g1_affine_t g1_from_bytes(const uint8_t in[96]) {
    if (in[0] & 0x40) return g1_affine_t::inf();
    return {fq_from_be(in), fq_from_be(in + 48)};
}
static void rand_scalar(uint8_t s[32]) {
    for (int i = 0; i < 32; i++) s[i] = (uint8_t)rng();
    s[31] &= 0x3f;
}
static void neg_scalar(const uint8_t s[32], uint8_t out[32]) {  // r - s
    static const uint32_t R[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                                  0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
    uint64_t bw = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t si;
        std::memcpy(&si, s + 4 * i, 4);
        uint64_t d = (uint64_t)R[i] - si - bw;
        uint32_t o = (uint32_t)d;
        std::memcpy(out + 4 * i, &o, 4);
        bw = (d >> 63) & 1;
    }
}

static bool same_point(const g1_xyzz_t &acc, const uint8_t expect[96]) {
    g1_affine_t a = xyzz_to_affine_inl(acc);
    uint8_t got[96];
    g1_to_bytes(a, got);
    return std::memcmp(got, expect, 96) == 0;
}

static void check_fields() {
    const fq32_t rinv = ref_rinv();
    for (int it = 0; it < 4000; it++) {
        fq_t a = rand_fq(), b = rand_fq(), c = rand_fq(), d = rand_fq();
        if (it < 96) {  // limb extremes (the column-sum bound) and zero
            if (it & 1) a = extreme_fq(it % 3);
            if (it & 2) b = extreme_fq((it / 3) % 3);
            if (it & 4) c = extreme_fq((it / 7) % 3);
            if (it & 8) d = extreme_fq((it / 11) % 3);
            if (it & 64) c = fq_t::zero();
        }
        const fq32_t va = ref_val(a), vb = ref_val(b), vc = ref_val(c), vd = ref_val(d);
        // Montgomery product / square / fused a b + c d against the plain integers, outputs normalised
        const fq_t ab = a * b, aa = sqr(a), ma = mul_add(a, b, c, d);
        CHECK(ref_eq(ref_val(ab), ref_mul(ref_mul(va, vb), rinv)), "mul it=%d", it);
        CHECK(ref_eq(ref_val(aa), ref_mul(ref_mul(va, va), rinv)), "sqr it=%d", it);
        CHECK(ref_eq(ref_val(ma), ref_mul(ref_add(ref_mul(va, vb), ref_mul(vc, vd)), rinv)), "mul_add it=%d", it);
        CHECK(normalised(ab) && normalised(aa) && normalised(ma), "product limbs not normalised it=%d", it);
        // output magnitude: |a b| / R + p / 2 < 0.6 p for operands below 3 p, so round(V / p) is -1, 0 or 1
        CHECK(fq_quot(ab) >= -1 && fq_quot(ab) <= 1 && fq_quot(ma) >= -1 && fq_quot(ma) <= 1, "product range it=%d", it);
        // add / sub / neg / x3 and the former lazy names
        CHECK(ref_eq(ref_val(a + b), ref_add(va, vb)) && normalised(a + b), "add it=%d", it);
        CHECK(ref_eq(ref_val(a - b), ref_sub(va, vb)) && normalised(a - b), "sub it=%d", it);
        CHECK(ref_eq(ref_val(-a), ref_sub(fq32_t::zero(), va)) && normalised(-a), "neg it=%d", it);
        CHECK(ref_eq(ref_val(fq_sub_lazy(a, b)), ref_sub(va, vb)), "sub_lazy it=%d", it);
        CHECK(ref_eq(ref_val(fq_neg_lazy(a)), ref_sub(fq32_t::zero(), va)), "neg_lazy it=%d", it);
        const fq_t x3 = fq_x3(a, b, c);
        CHECK(ref_eq(ref_val(x3), ref_sub(ref_sub(va, vb), ref_add(vc, vc))) && normalised(x3), "x3 it=%d", it);
        // is_zero / == modulo p for every representative; canonical form in [0, p)
        CHECK((a - a).is_zero() && fq_sub_kp(fq_t::zero(), (int32_t)(rng() % 9) - 4).is_zero(), "is_zero it=%d", it);
        CHECK(a.is_zero() == ref_eq(va, fq32_t::zero()), "is_zero value it=%d", it);
        CHECK(alt_rep(a) == a && !(a == a + fq_t::one()), "eq it=%d", it);
        const fq_t ca = fq_canon(a);
        CHECK(ref_eq(ref_val(ca), va) && fq_sign(ca) >= 0 && fq_sign(fq_sub_kp(ca, 1)) < 0, "canon it=%d", it);
        // the wire conversions round-trip
        CHECK(fq_from_raw(fq_to_raw(a)) == a, "raw round trip it=%d", it);
    }
}

// sums alone never grow without bound (the Miller loop's x3 = lambda^2 - 2 x): 400 doublings by addition and
// 400 x = x - 3 x steps stay normalised, bounded and equal to the integers mod p
static void check_growth() {
    fq_t a = rand_fq(), b = rand_fq();
    fq32_t va = ref_val(a), vb = ref_val(b);
    for (int it = 0; it < 400; it++) {
        a = a + a;
        va = ref_add(va, va);
        b = b - dbl(b) - b;
        vb = ref_sub(ref_sub(vb, ref_add(vb, vb)), vb);
        CHECK(normalised(a) && normalised(b) && a.v[12] <= (1 << 25) && a.v[12] >= -(1 << 25) &&
                  b.v[12] <= (1 << 25) && b.v[12] >= -(1 << 25), "growth not bounded it=%d", it);
    }
    CHECK(ref_eq(ref_val(a), va) && ref_eq(ref_val(b), vb), "growth values");
    CHECK(ref_eq(ref_val(a * b), ref_mul(ref_mul(va, vb), ref_rinv())), "growth product");
}

// the host-only 64-bit field (hostfield.h) against the device field: products, sums, inverses, and the host chains
// (scalar multiplication, window combination) against the generic group law over fq_t
static void check_host_field() {
    for (int it = 0; it < 2000; it++) {
        const fq_t a = rand_fq(), b = rand_fq();
        const host::hfq ha = host::to_h(a), hb = host::to_h(b);
        CHECK(host::from_h(ha * hb) == a * b && host::from_h(ha + hb) == a + b && host::from_h(ha - hb) == a - b,
              "hfq ops it=%d", it);
        CHECK(host::from_h(-ha) == -a && host::from_h(sqr(ha)) == sqr(a), "hfq neg/sqr it=%d", it);
        if (it < 20 && !a.is_zero()) CHECK(host::from_h(host::inverse_inl(ha)) * a == fq_t::one(), "hfq inverse it=%d", it);
    }
    uint8_t gen[96], gen2[192];
    or_g1_generator(gen);
    or_g2_generator(gen2);
    const g1_xyzz_t P = xyzz_dbl(xyzz_from_affine(g1_from_bytes(gen)));
    auto from2 = [](const uint8_t *p) -> g2_affine_t {
        return {{fq_from_be(p + 48), fq_from_be(p)}, {fq_from_be(p + 144), fq_from_be(p + 96)}};
    };
    const g2_xyzz_t Q = xyzz_dbl(xyzz_from_affine(from2(gen2)));
    for (int it = 0; it < 6; it++) {
        uint32_t k[8];
        for (auto &w : k) w = (uint32_t)rng();
        k[7] &= 0x3fffffff;
        const g1_affine_t a1 = xyzz_to_affine(host::xyzz_mul(P, k, 8)), b1 = xyzz_to_affine(xyzz_mul(P, k, 8));
        CHECK(a1.x == b1.x && a1.y == b1.y, "host g1 mul it=%d", it);
        const g2_affine_t a2 = xyzz_to_affine(host::xyzz_mul(Q, k, 8)), b2 = xyzz_to_affine(xyzz_mul(Q, k, 8));
        CHECK(a2.x == b2.x && a2.y == b2.y, "host g2 mul it=%d", it);
        std::vector<g1_xyzz_t> W;
        for (int w = 0; w < 5; w++) W.push_back(w == 2 ? g1_xyzz_t::inf() : xyzz_mul(P, k + w, 1));
        g1_xyzz_t ref = W.back();
        for (int w = 3; w >= 0; w--) {
            for (int i = 0; i < 13; i++) ref = xyzz_dbl(ref);
            ref = xyzz_add(ref, W[w]);
        }
        const g1_affine_t c1 = xyzz_to_affine(host::combine_windows(W, 13)), d1 = xyzz_to_affine(ref);
        CHECK(c1.x == d1.x && c1.y == d1.y, "host combine it=%d", it);
    }
}

static void check_g1_sequences() {
    uint8_t gen[96];
    or_g1_generator(gen);
    for (int seq = 0; seq < 200; seq++) {
        const int n = 1 + (int)(rng() % 24);
        g1_xyzz_t acc = g1_xyzz_t::inf();
        uint8_t expect[96];
        std::memset(expect, 0, 96);
        expect[0] = 0x40;
        uint8_t prev_s[32];
        bool have_prev = false;
        for (int i = 0; i < n; i++) {
            uint8_t s[32];
            const int kind = (int)(rng() % 8);
            if (kind == 0 && have_prev) std::memcpy(s, prev_s, 32);   // same point again: doubling branch
            else if (kind == 1 && have_prev) neg_scalar(prev_s, s);    // its negation: infinity branch
            else rand_scalar(s);
            const bool inf = kind == 2;
            const bool neg = rng() & 1;
            uint8_t pt[96];
            if (inf) {
                std::memset(pt, 0, 96);
                pt[0] = 0x40;
            } else {
                or_g1_mul(gen, s, pt);
            }
            g1_affine_t q = g1_from_bytes(pt);
            // other representatives of the coordinates of a point (an infinity stays the raw (0, 0) encoding:
            // curve.h coord_zero tests Fq infinity coordinates by their limbs)
            if (rng() & 1 && !q.is_inf()) q.x = alt_rep(q.x);
            if (rng() & 1 && !q.is_inf()) q.y = alt_rep(q.y);
            if (neg) q.y = lazy_neg(q.y);  // what k_accum_level0 does for a negative digit
            acc = xyzz_add_affine_inl(acc, q);
            if (!inf) {
                uint8_t term[96], sum[96];
                if (neg) {
                    uint8_t ns[32];
                    neg_scalar(s, ns);
                    or_g1_mul(gen, ns, term);
                } else {
                    std::memcpy(term, pt, 96);
                }
                or_g1_add(expect, term, sum);
                std::memcpy(expect, sum, 96);
                if (neg) neg_scalar(s, prev_s);  // prev_s = scalar of the point actually added
                else std::memcpy(prev_s, s, 32);
                have_prev = true;
            }
            CHECK(same_point(acc, expect), "g1 madd seq=%d step=%d kind=%d neg=%d", seq, i, kind, (int)neg);
        }
        // full XYZZ + XYZZ: acc + acc (doubling), acc + (-acc) (infinity), acc + fresh sum
        g1_xyzz_t d = xyzz_add_inl(acc, acc);
        uint8_t e2[96];
        or_g1_add(expect, expect, e2);
        CHECK(same_point(d, e2), "g1 add dbl seq=%d", seq);
        g1_xyzz_t z = xyzz_add_inl(acc, xyzz_neg(acc));
        CHECK(z.is_inf(), "g1 add inverse seq=%d", seq);
        uint8_t s[32], pt[96], e3[96];
        rand_scalar(s);
        or_g1_mul(gen, s, pt);
        g1_xyzz_t other = xyzz_add_affine_inl(g1_xyzz_t::inf(), g1_from_bytes(pt));
        other = xyzz_dbl_inl(other);
        uint8_t pt2[96];
        or_g1_add(pt, pt, pt2);
        or_g1_add(expect, pt2, e3);
        CHECK(same_point(xyzz_add_inl(acc, other), e3), "g1 add seq=%d", seq);
    }
}

// G2 through the generic (reduced) path the host uses for the window combination
static void check_g2() {
    uint8_t gen[192];
    or_g2_generator(gen);
    auto from = [](const uint8_t *p) -> g2_affine_t {
        if (p[0] & 0x40) return g2_affine_t::inf();
        return {{fq_from_be(p + 48), fq_from_be(p)}, {fq_from_be(p + 144), fq_from_be(p + 96)}};
    };
    for (int seq = 0; seq < 20; seq++) {
        g2_xyzz_t acc = g2_xyzz_t::inf();
        uint8_t expect[192];
        std::memset(expect, 0, 192);
        expect[0] = 0x40;
        for (int i = 0; i < 6; i++) {
            uint8_t s[32], pt[192], sum[192];
            rand_scalar(s);
            or_g2_mul(gen, s, pt);
            acc = xyzz_add_affine_inl(acc, from(pt));
            if (i == 3) acc = xyzz_add_affine_inl(acc, from(pt)), or_g2_add(expect, pt, sum), std::memcpy(expect, sum, 192);
            or_g2_add(expect, pt, sum);
            std::memcpy(expect, sum, 192);
        }
        g2_affine_t a = xyzz_to_affine_inl(acc), e = from(expect);
        CHECK(a.x == e.x && a.y == e.y, "g2 seq=%d", seq);
        // the bucket-reduction operations: full XYZZ additions (doubling and inverse branches too) and the
        // k_seg_fold double-and-add k * P
        uint8_t e2[192], ek[192], ks[32];
        or_g2_add(expect, expect, e2);
        g2_affine_t d = xyzz_to_affine_inl(xyzz_add_inl(acc, acc)), de = from(e2);
        CHECK(d.x == de.x && d.y == de.y, "g2 full add dbl seq=%d", seq);
        CHECK(xyzz_add_inl(acc, xyzz_neg(acc)).is_inf(), "g2 full add inverse seq=%d", seq);
        g2_affine_t d2 = xyzz_to_affine_inl(xyzz_dbl_inl(acc));
        CHECK(d2.x == de.x && d2.y == de.y, "g2 dbl seq=%d", seq);
        const uint32_t k = 1 + (uint32_t)(rng() % 5000000);
        std::memset(ks, 0, 32);
        std::memcpy(ks, &k, 4);
        or_g2_mul(expect, ks, ek);
        g2_xyzz_t m = acc;
        for (int bit = 30 - __builtin_clz(k); bit >= 0; bit--) {
            m = xyzz_dbl_inl(m);
            if ((k >> bit) & 1) m = xyzz_add_inl(m, acc);
        }
        g2_affine_t km = xyzz_to_affine_inl(m), kme = from(ek);
        CHECK(km.x == kme.x && km.y == kme.y, "g2 k*P seq=%d k=%u", seq, k);
    }
}

// GLV (glv.h): k = k1 + lambda k2 for random / edge / non-canonical scalars, and phi(P) = lambda P
static void words_of(const uint8_t *b, uint32_t *w, int n) {
    for (int i = 0; i < n; i++) std::memcpy(&w[i], b + 4 * i, 4);
}
static void check_glv() {
    static const uint32_t R[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                                  0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
    std::vector<std::vector<uint32_t>> ks;
    auto add = [&](std::initializer_list<uint32_t> w) {
        std::vector<uint32_t> v(w);
        v.resize(8, 0);
        ks.push_back(v);
    };
    add({0});
    add({1});
    add({GLV_LAMBDA[0] - 1, GLV_LAMBDA[1], GLV_LAMBDA[2], GLV_LAMBDA[3]});  // lambda - 1
    add({GLV_LAMBDA[0], GLV_LAMBDA[1], GLV_LAMBDA[2], GLV_LAMBDA[3]});      // lambda
    add({0, 0, 0, 0, 1});                                                   // 2^128
    add({R[0] - 1, R[1], R[2], R[3], R[4], R[5], R[6], R[7]});              // r - 1 = lambda^2 + lambda
    add({R[0], R[1], R[2], R[3], R[4], R[5], R[6], R[7]});                  // r (non-canonical: 0)
    add({R[0] + 5, R[1], R[2], R[3], R[4], R[5], R[6], R[7]});              // r + 5
    add({~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u});                          // 2^256 - 1
    for (int i = 0; i < 2000; i++) {
        std::vector<uint32_t> v(8);
        for (auto &x : v) x = (uint32_t)rng();
        v[7] &= (i & 1) ? 0x7fffffffu : 0x3fffffffu;
        ks.push_back(v);
    }
    for (size_t t = 0; t < ks.size(); t++) {
        uint32_t k[8], k1[4], k2[4];
        for (int i = 0; i < 8; i++) k[i] = ks[t][i];
        glv_split(k, k1, k2);
        // expected: k mod r (at most two subtractions: 2^256 < 3 r)
        uint32_t km[8];
        std::memcpy(km, k, sizeof(km));
        for (int j = 0; j < 2; j++)
            if (glv_geq(km, R, 8)) glv_sub(km, R, 8);
        // k1 + lambda k2 over 9 words
        uint32_t sum[9] = {0};
        for (int i = 0; i < 4; i++) {
            uint64_t carry = 0;
            for (int j = 0; j < 4; j++) {
                uint64_t cur = (uint64_t)sum[i + j] + (uint64_t)k2[i] * GLV_LAMBDA[j] + carry;
                sum[i + j] = (uint32_t)cur;
                carry = cur >> 32;
            }
            for (int j = i + 4; carry && j < 9; j++) {
                uint64_t cur = (uint64_t)sum[j] + carry;
                sum[j] = (uint32_t)cur;
                carry = cur >> 32;
            }
        }
        uint64_t carry = 0;
        for (int i = 0; i < 9; i++) {
            uint64_t cur = (uint64_t)sum[i] + (i < 4 ? k1[i] : 0) + carry;
            sum[i] = (uint32_t)cur;
            carry = cur >> 32;
        }
        bool eq = sum[8] == 0;
        for (int i = 0; i < 8; i++) eq = eq && sum[i] == km[i];
        CHECK(eq, "glv_split recombination t=%zu", t);
        CHECK(!glv_geq(k1, GLV_LAMBDA, 4), "glv_split k1 >= lambda t=%zu", t);
    }
    // phi(P) = lambda P on multiples of the generator (beta in the device's Montgomery form)
    uint8_t gen[96], lam[32] = {0};
    or_g1_generator(gen);
    std::memcpy(lam, GLV_LAMBDA, 16);
    const fq_t beta = glv_beta();
    for (int it = 0; it < 20; it++) {
        uint8_t s[32], pt[96], want[96], got[96];
        rand_scalar(s);
        or_g1_mul(gen, s, pt);
        or_g1_mul(pt, lam, want);
        g1_affine_t p = g1_from_bytes(pt);
        p.x = fq_canon(p.x * beta);
        g1_to_bytes(p, got);
        CHECK(std::memcmp(got, want, 96) == 0, "phi != lambda it=%d", it);
        // and on an XYZZ sum: phi(X, Y, ZZ, ZZZ) = (beta X, Y, ZZ, ZZZ)
        g1_xyzz_t acc = xyzz_dbl_inl(xyzz_add_affine_inl(g1_xyzz_t::inf(), g1_from_bytes(pt)));
        acc.X = acc.X * beta;
        uint8_t twice[96];
        or_g1_add(want, want, twice);
        CHECK(same_point(acc, twice), "phi on XYZZ it=%d", it);
    }
}

// the endomorphism membership tests of the checked key load (curve.h in_prime_subgroup_fast) against r P == O: on
// random multiples of the generators (members), and on on-curve points outside the subgroup -- random ones,
// cofactor-torsion points [r] Q and subgroup + torsion sums (subgroup_vectors.h)
static void check_subgroup_tests() {
    const SubgroupConsts sc = subgroup_consts();
    auto unhex = [](const char *h, uint8_t *out, int n) {
        for (int i = 0; i < n; i++) std::sscanf(h + 2 * i, "%2hhx", &out[i]);
    };
    auto g2from = [](const uint8_t *p) -> g2_affine_t {
        if (p[0] & 0x40) return g2_affine_t::inf();
        return {{fq_from_be(p + 48), fq_from_be(p)}, {fq_from_be(p + 144), fq_from_be(p + 96)}};
    };
    uint8_t g1g[96], g2g[192];
    or_g1_generator(g1g);
    or_g2_generator(g2g);
    for (int it = 0; it < 12; it++) {
        uint8_t s[32], p1[96], p2[192];
        rand_scalar(s);
        or_g1_mul(g1g, s, p1);
        or_g2_mul(g2g, s, p2);
        const g1_affine_t a1 = g1_from_bytes(p1);
        const g2_affine_t a2 = g2from(p2);
        CHECK(in_prime_subgroup(a1) && in_prime_subgroup_fast(a1, sc), "g1 member it=%d", it);
        CHECK(in_prime_subgroup(a2) && in_prime_subgroup_fast(a2, sc), "g2 member it=%d", it);
    }
    CHECK(in_prime_subgroup_fast(g1_affine_t::inf(), sc) && in_prime_subgroup_fast(g2_affine_t::inf(), sc), "inf");
    for (const char *h : G1_NON_SUBGROUP) {
        uint8_t b[96];
        unhex(h, b, 96);
        const g1_affine_t a = g1_from_bytes(b);
        CHECK(g1_on_curve(a) && !in_prime_subgroup(a) && !in_prime_subgroup_fast(a, sc), "g1 non-member %.16s", h + 80);
    }
    for (const char *h : G2_NON_SUBGROUP) {
        uint8_t b[192];
        unhex(h, b, 192);
        const g2_affine_t a = g2from(b);
        CHECK(g2_on_curve(a) && !in_prime_subgroup(a) && !in_prime_subgroup_fast(a, sc), "g2 non-member %.16s", h + 80);
    }
}

int main() {
    check_subgroup_tests();
    check_fields();
    check_growth();
    check_host_field();
    check_g1_sequences();
    check_g2();
    check_glv();
    if (failures) {
        std::printf("%d failures\n", failures);
        return 1;
    }
    std::printf("grouplaw OK\n");
    return 0;
}
