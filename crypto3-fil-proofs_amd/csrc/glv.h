// glv.h -- the GLV endomorphism of BLS12-381 G1 for the split-mode MSM ("GLV split").
//
// phi(x, y) = (beta x, y), beta a primitive cube root of unity in Fq, maps every point P of the r-torsion
// group to lambda P with lambda = z^2 - 1 (z = -0xd201000000010000 the BLS parameter; lambda^2 + lambda + 1
// = r, so lambda ~ 2^127.4).  A scalar k < r splits exactly as k = k1 + lambda k2 with k2 = floor(k /
// lambda), k1 = k mod lambda, both < 2^128, and k P = k1 P + k2 phi(P): the same two 128-bit half scalars
// as the 2^128 split (point i over P_i, point n + i over phi(P_i)) without a second base table.  In XYZZ
// coordinates phi(X, Y, ZZ, ZZZ) = (beta X, Y, ZZ, ZZZ), so phi costs one Fq multiplication and applies
// to a bucket SUM as well as to a point (sum_i phi(P_i) = phi(sum_i P_i)).
//
// beta is the root whose eigenvalue is this lambda (the other root, beta^2, acts as lambda^2 = -lambda - 1);
// tests/host/grouplaw_check.cpp checks phi(k G) = (lambda k) G against the oracle's scalar multiplication
// and the decomposition on random and edge scalars.
#pragma once
#include "field.h"

namespace mi {

constexpr uint32_t GLV_LAMBDA[4] = {0xffffffffu, 0x00000000u, 0x0001a402u, 0xac45a401u};
// floor(2^384 / lambda), 257 bits
constexpr uint32_t GLV_MU[9] = {0x896c72ddu, 0xda5e4f8du, 0x268bf7a3u, 0x389f49a7u, 0xf6cfee30u,
                                0x63f6e522u, 0xe01faaddu, 0x7c6becf1u, 0x00000001u};
// beta, canonical, little-endian 32-bit words
constexpr uint32_t GLV_BETA_RAW[12] = {0x0000aaacu, 0x8bfd0000u, 0x4f49fffdu, 0x409427ebu,
                                       0x0fb85f9bu, 0x897d2965u, 0x89759ad4u, 0xaa0d857du,
                                       0x63d4de85u, 0xec024086u, 0x397fe699u, 0x1a0111eau};

// a >= b over n words
MI_HD bool glv_geq(const uint32_t *a, const uint32_t *b, int n) {
    for (int i = n - 1; i >= 0; i--)
        if (a[i] != b[i]) return a[i] > b[i];
    return true;
}
// a -= b over n words (no borrow out: callers guarantee a >= b or want the value mod 2^(32 n))
MI_HD void glv_sub(uint32_t *a, const uint32_t *b, int n) {
    uint32_t borrow = 0;
    for (int i = 0; i < n; i++) {
        const uint64_t d = (uint64_t)a[i] - b[i] - borrow;
        a[i] = (uint32_t)d;
        borrow = (uint32_t)(d >> 63);
    }
}

// k (8 words, any value < 2^256; reduced mod r first) -> k1, k2 (4 words each) with
// k mod r = k1 + lambda k2, k1 < lambda, k2 <= (r - 1) / lambda.
MI_HD void glv_split(const uint32_t *kin, uint32_t *k1, uint32_t *k2) {
    uint32_t k[8];
    for (int i = 0; i < 8; i++) k[i] = kin[i];
    for (int t = 0; t < 2; t++)  // 2^256 < 3 r
        if (glv_geq(k, FrDesc::MOD, 8)) glv_sub(k, FrDesc::MOD, 8);
    // q = floor(k MU / 2^384) is floor(k / lambda) or one less (MU <= 2^384 / lambda < MU + 1, k < 2^384)
    uint32_t q[5] = {0, 0, 0, 0, 0};
    uint64_t lo = 0;
    uint32_t hi = 0;
    for (int j = 0; j < 17; j++) {  // product scanning, 96-bit column accumulator (lo + hi 2^64)
        for (int i = 0; i < 8; i++) {
            const int m = j - i;
            if (m < 0 || m > 8) continue;
            const uint64_t p = (uint64_t)k[i] * GLV_MU[m];
            lo += p;
            hi += lo < p;
        }
        if (j >= 12) q[j - 12] = (uint32_t)lo;
        lo = (lo >> 32) | ((uint64_t)hi << 32);
        hi = 0;
    }
    // r1 = k - q lambda over 5 words (the true remainder is < 2 lambda < 2^129)
    uint32_t ql[5];
    lo = 0;
    hi = 0;
    for (int j = 0; j < 5; j++) {  // low 5 words of q lambda
        for (int i = 0; i <= j; i++) {
            const int m = j - i;
            if (m > 3) continue;
            const uint64_t p = (uint64_t)q[i] * GLV_LAMBDA[m];
            lo += p;
            hi += lo < p;
        }
        ql[j] = (uint32_t)lo;
        lo = (lo >> 32) | ((uint64_t)hi << 32);
        hi = 0;
    }
    uint32_t r1[5] = {k[0], k[1], k[2], k[3], k[4]};
    glv_sub(r1, ql, 5);
    const uint32_t lam5[5] = {GLV_LAMBDA[0], GLV_LAMBDA[1], GLV_LAMBDA[2], GLV_LAMBDA[3], 0u};
    for (int t = 0; t < 2; t++)
        if (glv_geq(r1, lam5, 5)) {
            glv_sub(r1, lam5, 5);
            for (int i = 0; i < 5 && ++q[i] == 0; i++) {
            }
        }
    for (int i = 0; i < 4; i++) {
        k1[i] = r1[i];
        k2[i] = q[i];
    }
}

// beta in the device's Montgomery form
inline fq_t glv_beta() {
    fq32_t raw;
    for (int i = 0; i < 12; i++) raw.v[i] = GLV_BETA_RAW[i];
    return fq_from_raw(raw);
}

}  // namespace mi
