// poseidon_math.h -- Poseidon arithmetic shared by the kernels (poseidon.hip) and the host: Fr over
// 9 x 29-bit limbs, the permutation in its folded / sparse form, and the host derivation of the constant
// image.  Header-only so tests/host/poseidon_check.cpp runs the same code on the CPU.
// (The design notes are at the top of poseidon.hip.)
#pragma once
#include <stdexcept>
#include <cstdlib>
#include <utility>
#include <vector>

#include "field.h"
#include "fr29.h"
#include "poseidon.h"

namespace mi {

// ---------------------------------------------------------------------------------------------
// Fr over 9 x 29-bit limbs
// ---------------------------------------------------------------------------------------------
// row . s over T terms: chunks of <= 6 products per reduction, sums lazily added (each chunk < 1.5r
// for rows < r and s < 5r, so T <= 12 gives < 3r)
template <int T>
MI_HD fr29_t fr29_row(const fr29_t *row, const fr29_t *s) {
    if constexpr (T <= 6) {
        return fr29_dot<T>(row, s);
    } else {
        constexpr int A = (T + 1) / 2;
        return fr29_add(fr29_row<A>(row, s), fr29_row<T - A>(row + A, s + A));
    }
}

// ---------------------------------------------------------------------------------------------
// constants (host derivation) and their device image
// ---------------------------------------------------------------------------------------------
namespace pos_detail {

// Filecoin / neptune "Standard" round numbers (R_F, R_P) per arity
inline bool round_numbers(unsigned arity, int &rf, int &rp) {
    switch (arity) {
        case 2: rf = 8, rp = 55; return true;
        case 4: rf = 8, rp = 56; return true;
        case 8: rf = 8, rp = 57; return true;
        case 11: rf = 8, rp = 57; return true;
        default: return false;
    }
}

// Grain LFSR of the Poseidon reference parameter script, self-shrinking output
struct Grain {
    uint8_t st[80];
    int pos = 0;  // st is a ring: bit i of the window is st[(pos + i) % 80]
    explicit Grain(const std::vector<uint8_t> &seed) {
        for (int i = 0; i < 80; i++) st[i] = seed[i];
        for (int i = 0; i < 160; i++) step();
    }
    uint8_t bit(int i) const { return st[(pos + i) % 80]; }
    uint8_t step() {
        const uint8_t b = bit(62) ^ bit(51) ^ bit(38) ^ bit(23) ^ bit(13) ^ bit(0);
        st[pos] = b;  // the oldest bit leaves, the new one enters at the end of the window
        pos = (pos + 1) % 80;
        return b;
    }
    uint8_t next() {
        for (;;) {
            const uint8_t b1 = step(), b2 = step();
            if (b1) return b2;
        }
    }
};

// r as 32-bit words (canonical comparison of the candidates)
inline bool below_r(const uint32_t w[8]) {
    for (int i = 7; i >= 0; i--)
        if (w[i] != FrDesc::MOD[i]) return w[i] < FrDesc::MOD[i];
    return false;
}

inline std::vector<fr_t> grain_constants(unsigned t, int rf, int rp, unsigned sbox_field) {
    std::vector<uint8_t> seed;
    auto app = [&](int n, uint64_t v) {
        for (int i = n - 1; i >= 0; i--) seed.push_back((v >> i) & 1);
    };
    app(2, 1);           // prime field
    app(4, sbox_field);  // S-box field of the LFSR seed
    app(12, 255);        // field size in bits
    app(12, t);
    app(10, (uint64_t)rf);
    app(10, (uint64_t)rp);
    app(30, (1u << 30) - 1);
    Grain g(seed);
    std::vector<fr_t> out;
    const size_t need = (size_t)(rf + rp) * t;
    while (out.size() < need) {
        uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int b = 254; b >= 0; b--)  // most significant bit first
            if (g.next()) w[b >> 5] |= 1u << (b & 31);
        if (!below_r(w)) continue;
        fr_t raw;
        for (int i = 0; i < 8; i++) raw.v[i] = w[i];
        out.push_back(to_mont(raw));
    }
    return out;
}

inline fr_t fr_small(uint64_t v) {
    fr_t raw = fr_t::zero();
    raw.v[0] = (uint32_t)v;
    raw.v[1] = (uint32_t)(v >> 32);
    return to_mont(raw);
}

using Mat = std::vector<std::vector<fr_t>>;
inline Mat mat_mul(const Mat &a, const Mat &b) {
    const size_t n = a.size(), m = b[0].size(), k = b.size();
    Mat r(n, std::vector<fr_t>(m, fr_t::zero()));
    for (size_t i = 0; i < n; i++)
        for (size_t j = 0; j < m; j++) {
            fr_t s = fr_t::zero();
            for (size_t q = 0; q < k; q++) s = s + a[i][q] * b[q][j];
            r[i][j] = s;
        }
    return r;
}
inline Mat mat_inv(Mat a) {  // Gauss-Jordan over Fr
    const size_t n = a.size();
    Mat inv(n, std::vector<fr_t>(n, fr_t::zero()));
    for (size_t i = 0; i < n; i++) inv[i][i] = fr_t::one();
    for (size_t c = 0; c < n; c++) {
        size_t p = c;
        while (p < n && a[p][c].is_zero()) p++;
        if (p == n) throw std::logic_error("poseidon: singular MDS sub-matrix");
        std::swap(a[p], a[c]);
        std::swap(inv[p], inv[c]);
        const fr_t iv = inverse(a[c][c]);
        for (size_t j = 0; j < n; j++) {
            a[c][j] = a[c][j] * iv;
            inv[c][j] = inv[c][j] * iv;
        }
        for (size_t r = 0; r < n; r++) {
            if (r == c || a[r][c].is_zero()) continue;
            const fr_t f = a[r][c];
            for (size_t j = 0; j < n; j++) {
                a[r][j] = a[r][j] - f * a[c][j];
                inv[r][j] = inv[r][j] - f * inv[c][j];
            }
        }
    }
    return inv;
}

}  // namespace pos_detail

// S-box field of the Grain LFSR seed: 1, the value Filecoin's Poseidon seeds it with (oracle/poseidon_ref.py
// SBOX_FIELD).  A fixed constant: nothing at run time changes the round constants (and with them every tree root).
constexpr unsigned kPoseidonSboxField = 1;
inline constexpr unsigned poseidon_sbox_field() { return kPoseidonSboxField; }

// Host-side derivation of the device constant image (layout in poseidon.h: PosK offsets).
inline PoseidonHost poseidon_derive(unsigned arity, unsigned sbox_field) {
    using namespace pos_detail;
    PoseidonHost h;
    int rf = 0, rp = 0;
    if (!round_numbers(arity, rf, rp)) throw std::invalid_argument("poseidon: arity must be 2, 4, 8 or 11");
    const unsigned t = arity + 1;
    h.arity = arity;
    h.t = t;
    h.rf = rf;
    h.rp = rp;
    std::vector<fr_t> rc = grain_constants(t, rf, rp, sbox_field);
    // Cauchy MDS: M[i][j] = 1 / (i + t + j)  (symmetric)
    Mat M(t, std::vector<fr_t>(t));
    for (unsigned i = 0; i < t; i++)
        for (unsigned j = 0; j < t; j++) M[i][j] = inverse(fr_small(i + t + j));
    // fold the constants of elements 1.. of every partial round forward into the next round
    const int half = rf / 2;
    auto c = [&](int rnd, unsigned i) -> fr_t & { return rc[(size_t)rnd * t + i]; };
    for (int rnd = half; rnd < half + rp; rnd++) {
        for (unsigned i = 0; i < t; i++) {
            fr_t add = fr_t::zero();
            for (unsigned j = 1; j < t; j++) add = add + M[i][j] * c(rnd, j);
            c(rnd + 1, i) = c(rnd + 1, i) + add;
        }
        for (unsigned j = 1; j < t; j++) c(rnd, j) = fr_t::zero();
    }
    // sparse factorisation of the partial rounds
    const unsigned u = t - 1;
    Mat Mh(u, std::vector<fr_t>(u)), Ah(u, std::vector<fr_t>(u, fr_t::zero()));
    std::vector<fr_t> v(u), w(u);
    for (unsigned i = 0; i < u; i++) {
        v[i] = M[0][i + 1];
        w[i] = M[i + 1][0];
        Ah[i][i] = fr_t::one();
        for (unsigned j = 0; j < u; j++) Mh[i][j] = M[i + 1][j + 1];
    }
    const Mat Mh_inv = mat_inv(Mh);
    std::vector<fr_t> wk = w;
    std::vector<fr_t> sparse;  // per sparse round: row (t entries) then w^ (t - 1 entries)
    for (int k = 1; k < rp; k++) {
        sparse.push_back(M[0][0]);
        for (unsigned j = 0; j < u; j++) {  // (v^T A^_{k-1})_j
            fr_t s = fr_t::zero();
            for (unsigned q = 0; q < u; q++) s = s + v[q] * Ah[q][j];
            sparse.push_back(s);
        }
        Ah = mat_mul(Mh, Ah);  // A^_k
        std::vector<fr_t> nw(u);  // w^_k = M^^-1 w^_{k-1}
        for (unsigned i = 0; i < u; i++) {
            fr_t s = fr_t::zero();
            for (unsigned q = 0; q < u; q++) s = s + Mh_inv[i][q] * wk[q];
            nw[i] = s;
        }
        wk = nw;
        for (unsigned j = 0; j < u; j++) sparse.push_back(wk[j]);
    }
    // last partial round: dense M A_{R_P - 1}
    Mat A(t, std::vector<fr_t>(t, fr_t::zero()));
    A[0][0] = fr_t::one();
    for (unsigned i = 0; i < u; i++)
        for (unsigned j = 0; j < u; j++) A[i + 1][j + 1] = Ah[i][j];
    const Mat N = mat_mul(M, A);

    auto put = [&](const fr_t &x) { h.img.push_back(fr29_from_fr(x)); };
    h.off_tag = h.img.size();
    put(fr_small((1ull << arity) - 1));
    fr_t r2;
    for (int i = 0; i < 8; i++) r2.v[i] = FrDesc::R2[i];
    put(r2);  // R^2 mod r: a raw input times it (one REDC) is the input in Montgomery form
    h.off_rc_first = h.img.size();
    for (int rnd = 0; rnd < half; rnd++)
        for (unsigned i = 0; i < t; i++) put(c(rnd, i));
    h.off_rc_part = h.img.size();
    for (int rnd = half; rnd < half + rp; rnd++) put(c(rnd, 0));
    h.off_rc_last = h.img.size();
    for (int rnd = half + rp; rnd < rf + rp; rnd++)
        for (unsigned i = 0; i < t; i++) put(c(rnd, i));
    h.off_mds = h.img.size();
    for (unsigned i = 0; i < t; i++)
        for (unsigned j = 0; j < t; j++) put(M[i][j]);
    h.off_sparse = h.img.size();
    for (const fr_t &x : sparse) put(x);
    h.off_dense = h.img.size();
    for (unsigned i = 0; i < t; i++)
        for (unsigned j = 0; j < t; j++) put(N[i][j]);
    // the plain (unfolded) constants and MDS, canonical, for mi_poseidon_constants
    std::vector<fr_t> raw_rc = grain_constants(t, rf, rp, sbox_field);
    for (auto &x : raw_rc) h.plain_rc.push_back(from_mont(x));
    for (unsigned i = 0; i < t; i++)
        for (unsigned j = 0; j < t; j++) h.plain_mds.push_back(from_mont(M[i][j]));
    return h;
}

// ---------------------------------------------------------------------------------------------
// device permutation
// ---------------------------------------------------------------------------------------------
// compile-time loop over I = 0 .. N-1: the state arrays are indexed by constants only, so they stay in
// registers (a `#pragma unroll` loop whose body holds three Montgomery products was left rolled by the
// unroller and the state went to scratch memory)
template <class F, int... I>
MI_HD void sfor_impl(F &&f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
MI_HD void sfor(F &&f) {
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}

template <int T>
MI_HD void mat_apply(fr29_t (&s)[T], const fr29_t *__restrict__ m) {
    fr29_t n[T];
    sfor<T>([&](auto i) { n[i] = fr29_row<T>(m + i * T, s); });
    sfor<T>([&](auto i) { s[i] = n[i]; });
}

template <int T>
MI_HD void full_round(fr29_t (&s)[T], const fr29_t *__restrict__ rc,
                                           const fr29_t *__restrict__ m) {
    sfor<T>([&](auto i) { s[i] = fr29_sbox(fr29_add(s[i], rc[i])); });
    mat_apply<T>(s, m);
}

template <int T>
MI_HD fr29_t poseidon_permute(fr29_t (&s)[T], const PosK &k) {
    const fr29_t *img = k.img;
    const fr29_t *mds = img + k.off_mds;
#pragma unroll 1
    for (int r = 0; r < k.rf / 2; r++) full_round<T>(s, img + k.off_rc_first + r * T, mds);
    const fr29_t *sp = img + k.off_sparse;
#pragma unroll 1
    for (int q = 0; q < k.rp - 1; q++, sp += 2 * T - 1) {
        s[0] = fr29_sbox(fr29_add(s[0], img[k.off_rc_part + q]));
        const fr29_t n0 = fr29_row<T>(sp, s);
        sfor<T - 1>([&](auto j) {  // element j + 1, stays < 4r
            s[j + 1] = fr29_sub_if_ge(fr29_add(s[j + 1], fr29_mul(sp[T + j], s[0])), R2X29);
        });
        s[0] = n0;
    }
    s[0] = fr29_sbox(fr29_add(s[0], img[k.off_rc_part + k.rp - 1]));
    mat_apply<T>(s, img + k.off_dense);
#pragma unroll 1
    for (int r = 0; r < k.rf / 2; r++) full_round<T>(s, img + k.off_rc_last + r * T, mds);
    return s[1];
}

// one hash on the host with the device arithmetic (tests: tests/host/poseidon_check.cpp)
inline fr_t poseidon_hash_host(const PoseidonHost &h, const fr_t *x) {
    PosK k{h.img.data(), h.rf, h.rp, (uint32_t)h.off_tag, (uint32_t)h.off_rc_first, (uint32_t)h.off_rc_part,
           (uint32_t)h.off_rc_last, (uint32_t)h.off_mds, (uint32_t)h.off_sparse, (uint32_t)h.off_dense};
    auto run = [&](auto tt) -> fr_t {
        constexpr int T = decltype(tt)::value;
        fr29_t s[T];
        s[0] = k.img[k.off_tag];
        for (int j = 1; j < T; j++) s[j] = fr29_mul(fr29_from_fr(x[j - 1]), k.img[k.off_tag + 1]);
        return fr_from_fr29(fr29_from_mont(poseidon_permute<T>(s, k)));
    };
    switch (h.arity) {
        case 2: return run(std::integral_constant<int, 3>{});
        case 4: return run(std::integral_constant<int, 5>{});
        case 8: return run(std::integral_constant<int, 9>{});
        case 11: return run(std::integral_constant<int, 12>{});
        default: throw std::invalid_argument("poseidon: arity must be 2, 4, 8 or 11");
    }
}


}  // namespace mi
