// stacked_pos_check.cpp -- TEST INFRASTRUCTURE: the stacked witness's Poseidon gadget emission
// (csrc/stacked_pos.h pos_run on the production 29-bit sparse permutation) run on the host, against a literal
// evaluation of the same gadget variables (state * M per round, every S-box input v, v^2, v^4, v^5 in plain
// Montgomery fr_t; the layout of oracle/stacked_circuit.py poseidon_hash_circuit).
// stdin: lines "arity x_1 .. x_arity" (hex); stdout: per line the number of variables and "ok" or the first
// mismatching variable index.
#include <cstdio>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "poseidon_math.h"
#include "prover.h"
#include "stacked_pos.h"

using namespace mi;

static fr_t fr_from_hex(const std::string &h) {
    fr_t r = fr_t::zero();
    int bit = 0;
    for (int i = (int)h.size() - 1; i >= 0 && bit < 256; i--, bit += 4) {
        const char ch = h[i];
        const uint32_t d = ch <= '9' ? ch - '0' : (ch | 32) - 'a' + 10;
        r.v[bit >> 5] |= d << (bit & 31);
    }
    return r;
}

struct VecSink {
    std::vector<fr_t> v;
    void put(const fr29_t &x) { v.push_back(fr_from_fr29(fr29_from_mont(x))); }
};

// literal gadget variables in Montgomery fr_t
static std::vector<fr_t> literal(const PoseidonHost &h, const fr_t *x) {
    const unsigned t = h.t;
    std::vector<fr_t> rc, m, s(t), out;
    for (auto &c : h.plain_rc) rc.push_back(to_mont(c));
    for (auto &c : h.plain_mds) m.push_back(to_mont(c));
    s[0] = pos_detail::fr_small((1ull << h.arity) - 1);
    for (unsigned j = 1; j < t; j++) s[j] = to_mont(x[j - 1]);
    const int half = h.rf / 2;
    size_t k = 0;
    for (int rnd = 0; rnd < h.rf + h.rp; rnd++) {
        for (unsigned i = 0; i < t; i++) s[i] = s[i] + rc[k + i];
        k += t;
        const bool full = rnd < half || rnd >= half + h.rp;
        for (unsigned i = 0; i < (full ? t : 1u); i++) {
            const fr_t v = s[i], v2 = v * v, v4 = v2 * v2, v5 = v4 * v;
            if (!(rnd == 0 && i == 0)) {
                if (rnd > 0) out.push_back(from_mont(v));
                out.push_back(from_mont(v2));
                out.push_back(from_mont(v4));
                out.push_back(from_mont(v5));
            }
            s[i] = v5;
        }
        std::vector<fr_t> n(t, fr_t::zero());
        for (unsigned j = 0; j < t; j++)
            for (unsigned i = 0; i < t; i++) n[j] = n[j] + s[i] * m[i * t + j];
        s = n;
    }
    out.push_back(from_mont(s[1]));
    return out;
}

template <int T>
static std::vector<fr_t> fast(const PoseidonHost &h, const fr_t *x) {
    PosK k{h.img.data(), h.rf, h.rp, (uint32_t)h.off_tag, (uint32_t)h.off_rc_first, (uint32_t)h.off_rc_part,
           (uint32_t)h.off_rc_last, (uint32_t)h.off_mds, (uint32_t)h.off_sparse, (uint32_t)h.off_dense};
    fr29_t s[T];
    s[0] = k.img[k.off_tag];
    for (int j = 1; j < T; j++) s[j] = fr29_mul(fr29_from_fr(x[j - 1]), k.img[k.off_tag + 1]);
    VecSink sink;
    stacked::pos_run<T, VecSink>(k, s, &sink);
    return sink.v;
}

int main() {
    std::map<unsigned, PoseidonHost> tabs;
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        unsigned arity;
        if (!(in >> arity)) continue;
        if (!tabs.count(arity)) tabs[arity] = poseidon_derive(arity, poseidon_sbox_field());
        const PoseidonHost &h = tabs[arity];
        fr_t x[16];
        for (unsigned j = 0; j < arity; j++) {
            std::string hx;
            in >> hx;
            x[j] = fr_from_hex(hx);
        }
        std::vector<fr_t> a = literal(h, x), b;
        switch (arity) {
            case 2: b = fast<3>(h, x); break;
            case 4: b = fast<5>(h, x); break;
            case 8: b = fast<9>(h, x); break;
            default: b = fast<12>(h, x); break;
        }
        size_t bad = a.size() == b.size() ? a.size() : std::min(a.size(), b.size());
        for (size_t i = 0; i < std::min(a.size(), b.size()); i++)
            if (!(a[i] == b[i])) {
                bad = i;
                break;
            }
        if (a.size() == b.size() && bad == a.size())
            printf("%zu ok\n", a.size());
        else
            printf("%zu mismatch at %zu (fast emitted %zu)\n", a.size(), bad, b.size());
    }
    return 0;
}
