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

int main() {
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
