// tree_c.cpp -- the tree C / tree R-last calls a generate_tree_c_gpu / generate_tree_r_last port would make,
// through the C++ host layer (include/mi355x_groth16.hpp).  Deterministic labels (SplitMix64, < 2^252 so
// canonical); prints the tree C root, the last cached tree R-last row and the replica's first node (hex).
//   tree_c <log8_nodes>
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

static void hex(const uint8_t *p) {
    for (int i = 31; i >= 0; i--) std::printf("%02x", p[i]);
    std::printf("\n");
}

int main(int argc, char **argv) {
    const int lg8 = argc > 1 ? std::atoi(argv[1]) : 3;
    uint64_t nodes = 1;
    for (int i = 0; i < lg8; i++) nodes *= 8;
    uint64_t seed = 42;
    auto labels = [&](size_t n) {
        std::vector<uint8_t> v(32 * n);
        for (size_t i = 0; i < 4 * n; i++) {
            uint64_t w = splitmix(seed);
            if (i % 4 == 3) w &= 0x0FFFFFFFFFFFFFFFull;
            for (int b = 0; b < 8; b++) v[8 * i + b] = (uint8_t)(w >> (8 * b));
        }
        return v;
    };
    try {
        mi355x::context ctx(0);
        std::vector<std::vector<uint8_t>> layers;
        std::vector<const uint8_t *> ptrs;
        for (int l = 0; l < 11; l++) layers.push_back(labels(nodes));
        for (auto &l : layers) ptrs.push_back(l.data());
        auto bt = mi355x::column_tree_builder(ctx, 11, 8).add_final_columns(ptrs, nodes);
        hex(bt.second.data() + bt.second.size() - 32);  // root
        std::vector<uint8_t> data = labels(nodes);
        auto tr = mi355x::generate_tree_r_last(ctx, nodes, layers[10].data(), data.data(), 8, 0);
        hex(tr.data() + tr.size() - 32);
        hex(data.data());
    } catch (const mi355x::error &e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
