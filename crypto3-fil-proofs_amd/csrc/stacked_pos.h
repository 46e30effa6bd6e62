// stacked_pos.h -- the Poseidon gadget's witness from the production permutation (host + device).
//
// The production permutation (poseidon_math.h: 9 x 29-bit lazy Montgomery limbs, folded constants, sparse
// partial rounds) has the literal permutation's S-box inputs: the full rounds are literal, and in the
// partial rounds the sparse factorisation keeps element 0 in the literal basis with its folded constant equal
// to the literal one (A_k = diag(1, M^k)).  The gadget's variables (oracle/stacked_circuit.py
// poseidon_hash_circuit: per S-box after the first round its input v, then v^2, v^4, v^5; first-round S-boxes
// of the inputs without v; the domain tag's first S-box constant; finally the digest) are functions of those
// inputs only, so pos_run emits them to a Sink as it goes.  tests/host/stacked_pos_check.cpp runs this on
// the host against a literal evaluation of the same variables.
#pragma once
#include "poseidon_math.h"

namespace mi {
namespace stacked {

template <int T, class Sink>
MI_HD fr29_t pos_run(const PosK &k, fr29_t (&s)[T], Sink *E) {
    const fr29_t *img = k.img;
    const fr29_t *mds = img + k.off_mds;
    // one S-box on input x; `first`: a first-round S-box (its input is a linear combination, not allocated)
    auto sbox = [&](const fr29_t &x, bool first) -> fr29_t {
        const fr29_t x2 = fr29_sqr(x), x4 = fr29_sqr(x2), x5 = fr29_mul(x4, x);
        if (E) {
            if (!first) E->put(x);
            E->put(x2);
            E->put(x4);
            E->put(x5);
        }
        return x5;
    };
    const int half = k.rf / 2;
    for (int r = 0; r < half; r++) {
        const fr29_t *rc = img + k.off_rc_first + r * T;
        sfor<T>([&](auto i) {
            const fr29_t x = fr29_add(s[i], rc[i]);
            s[i] = (r == 0 && i == 0) ? fr29_sbox(x) : sbox(x, r == 0);  // the domain tag's first S-box: constant
        });
        mat_apply<T>(s, mds);
    }
    const fr29_t *sp = img + k.off_sparse;
    for (int q = 0; q < k.rp - 1; q++, sp += 2 * T - 1) {
        s[0] = sbox(fr29_add(s[0], img[k.off_rc_part + q]), false);
        const fr29_t n0 = fr29_row<T>(sp, s);
        sfor<T - 1>([&](auto j) { s[j + 1] = fr29_sub_if_ge(fr29_add(s[j + 1], fr29_mul(sp[T + j], s[0])), R2X29); });
        s[0] = n0;
    }
    s[0] = sbox(fr29_add(s[0], img[k.off_rc_part + k.rp - 1]), false);
    mat_apply<T>(s, img + k.off_dense);
    for (int r = 0; r < half; r++) {
        const fr29_t *rc = img + k.off_rc_last + r * T;
        sfor<T>([&](auto i) { s[i] = sbox(fr29_add(s[i], rc[i]), false); });
        mat_apply<T>(s, mds);
    }
    if (E) E->put(s[1]);
    return s[1];
}

}  // namespace stacked
}  // namespace mi
