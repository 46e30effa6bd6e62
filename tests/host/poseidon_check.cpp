// poseidon_check.cpp -- TEST INFRASTRUCTURE: the device Poseidon arithmetic (csrc/poseidon.hip: 9 x 29-bit
// lazy Fr, folded round constants, sparse partial rounds) run on the host, for a CPU check against the
// literal restatement oracle/poseidon_ref.py (tests/test_cpu_poseidon.py).
// stdin: lines "arity x_1 .. x_arity" (hex); stdout: one hex digest per line.
#include <cstdio>
#include <cstring>
#include <iostream>
#include <map>
#include <sstream>
#include <string>

#include "poseidon_math.h"
#include "prover.h"

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

// fr29_dot_lat (the latency-bound witness kernels' product) against fr29_dot: the same integer for K = 1 .. 6 terms
// over random carry-normalised operands below 8r, and the edge operands 0, 1, r - 1, 8r - 1
template <int K>
static bool check_dot_lat(uint64_t &seed) {
    auto rnd = [&] {
        seed ^= seed << 13, seed ^= seed >> 7, seed ^= seed << 17;
        return seed;
    };
    for (int it = 0; it < 20000; it++) {
        fr29_t a[K], b[K];
        for (int q = 0; q < K; q++) {
            for (int l = 0; l < 9; l++) a[q].v[l] = (uint32_t)rnd() & M29, b[q].v[l] = (uint32_t)rnd() & M29;
            a[q].v[8] &= (1u << 26) - 1, b[q].v[8] &= (1u << 26) - 1;  // < 2^258 (~8r)
            const int kind = (int)(rnd() % 8);
            if (kind == 0) std::memset(&a[q], 0, sizeof a[q]);
            if (kind == 1) for (int l = 0; l < 9; l++) a[q].v[l] = l == 0;
            if (kind == 2) for (int l = 0; l < 9; l++) a[q].v[l] = FrDesc::MOD29[l] - (l == 0);
            if (kind == 3) for (int l = 0; l < 9; l++) b[q].v[l] = l < 8 ? M29 : (1u << 26) - 1;
        }
        const fr29_t x = fr29_dot<K>(a, b), y = fr29_dot_lat<K>(a, b);
        if (std::memcmp(&x, &y, sizeof x) != 0) {
            std::printf("fr29_dot_lat<%d> differs at iteration %d\n", K, it);
            return false;
        }
    }
    return true;
}

int main(int argc, char **argv) {
    if (argc > 1 && std::strcmp(argv[1], "lat") == 0) {
        uint64_t seed = 0x9E3779B97F4A7C15ull;
        const bool ok = check_dot_lat<1>(seed) && check_dot_lat<2>(seed) && check_dot_lat<3>(seed) &&
                        check_dot_lat<4>(seed) && check_dot_lat<5>(seed) && check_dot_lat<6>(seed);
        std::printf(ok ? "dot_lat OK\n" : "dot_lat FAILED\n");
        return ok ? 0 : 1;
    }
    std::map<unsigned, PoseidonHost> tabs;
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        unsigned arity;
        if (!(in >> arity)) continue;
        if (!tabs.count(arity)) tabs[arity] = poseidon_derive(arity, poseidon_sbox_field());
        fr_t x[16];
        for (unsigned j = 0; j < arity; j++) {
            std::string h;
            in >> h;
            x[j] = fr_from_hex(h);
        }
        const fr_t d = poseidon_hash_host(tabs[arity], x);
        for (int i = 7; i >= 0; i--) std::printf("%08x", d.v[i]);
        std::printf("\n");
    }
    return 0;
}
