// sdr_labels.cpp -- the labelling-proof calls a prove_layers port would make (vanilla/proof.hpp:190-255),
// through the C++ host layer (include/mi355x_groth16.hpp).  Deterministic inputs (SplitMix64): `count`
// labels over 14 parents each at layers 2..11, then one labeling_proof (37 repeated parents) verified
// against its own label.  Prints every label (hex, byte 0 first) and "verify ok".
//   sdr_labels <count>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mi355x_groth16.hpp"

static uint64_t splitmix(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char **argv) {
    const size_t count = argc > 1 ? (size_t)std::atoi(argv[1]) : 8;
    uint64_t seed = 7;
    auto fr = [&]() {
        mi355x::fr32 v;
        for (int w = 0; w < 4; w++) {
            const uint64_t x = splitmix(seed);
            for (int b = 0; b < 8; b++) v[8 * w + b] = (uint8_t)(x >> (8 * b));
        }
        return v;
    };
    try {
        mi355x::context ctx(0);
        const mi355x::fr32 replica_id = fr();
        std::vector<std::uint32_t> layers(count);
        std::vector<std::uint64_t> nodes(count);
        std::vector<mi355x::fr32> parents(14 * count);
        for (size_t i = 0; i < count; i++) {
            layers[i] = 2 + (uint32_t)(i % 10);
            nodes[i] = 1 + splitmix(seed) % (1ull << 30);
        }
        for (auto &p : parents) p = fr();
        const auto labels = mi355x::create_labels(ctx, replica_id, layers, nodes, parents, 14);
        for (const auto &l : labels) {
            for (int b = 0; b < 32; b++) std::printf("%02x", l[b]);
            std::printf("\n");
        }
        mi355x::labeling_proof lp;
        for (int k = 0; k < 37; k++) lp.parents.push_back(parents[k % 14]);
        lp.layer_index = layers[0];
        lp.node = nodes[0];
        if (!lp.verify(ctx, replica_id, labels[0])) {
            std::fprintf(stderr, "labeling proof does not verify\n");
            return 1;
        }
        std::printf("verify ok\n");
    } catch (const mi355x::error &e) {
        std::fprintf(stderr, "error %d: %s\n", e.code, e.what());
        return 2;
    }
    return 0;
}
