// prove_synthetic.cpp -- C++ host example over include/mi355x_groth16.hpp: builds a synthetic
// R1CS (mi_synth), generates a proving key on the GPU from fixed toxic waste, and runs the
// compound_proof::circuit_proofs partition loop, self-verifies the MultiProof (api/seal.hpp:310-313)
// and prints one hex proof per partition.
//
//   g++ -std=c++17 -I../../include prove_synthetic.cpp -L../build -lfilgpu -o prove_synthetic
//   ./prove_synthetic <log_rows> <partitions>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "mi355x_groth16.hpp"

int main(int argc, char **argv) {
    unsigned log_rows = argc > 1 ? atoi(argv[1]) : 10;
    int parts = argc > 2 ? atoi(argv[2]) : 2;
    try {
        mi_synth *syn = nullptr;
        mi355x::check(mi_synth_generate(log_rows, 4, 1, &syn));
        mi_r1cs cs;
        mi355x::check(mi_synth_r1cs(syn, &cs));
        const uint8_t *zp = nullptr;
        uint64_t nv = 0;
        mi355x::check(mi_synth_witness(syn, &zp, &nv));
        std::vector<mi355x::fr32> z(nv);
        memcpy(z.data(), zp, 32 * nv);

        mi355x::context ctx(0);
        mi355x::circuit circ(ctx, cs);
        std::array<mi355x::fr32, 5> toxic{};
        for (int i = 0; i < 5; i++) toxic[i][0] = (uint8_t)(11 + i);  // tau=11, alpha=12, ...
        auto pk = mi355x::proving_key::generate(ctx, circ, toxic);
        std::vector<std::vector<mi355x::fr32>> assignments(parts, z);
        std::vector<std::pair<mi355x::fr32, mi355x::fr32>> blind(parts);
        for (int k = 0; k < parts; k++) {
            blind[k].first = {};
            blind[k].second = {};
            blind[k].first[0] = (uint8_t)(100 + k);
            blind[k].second[0] = (uint8_t)(200 + k);
        }
        mi355x::multi_proof mp = mi355x::circuit_proofs(ctx, pk, circ, assignments, blind);
        // seal_commit_phase2 never returns a proof that does not verify (api/seal.hpp:310-313)
        std::vector<std::vector<mi355x::fr32>> inputs(parts);
        for (int k = 0; k < parts; k++) inputs[k].assign(z.begin() + 1, z.begin() + cs.num_inputs);
        if (!mp.verify(inputs)) {
            fprintf(stderr, "post-seal verification sanity check failed\n");
            return 2;
        }
        // the production form: blinding drawn inside the library (internal randomness)
        mi355x::multi_proof mr = mi355x::circuit_proofs(ctx, pk, circ, assignments);
        if (!mr.verify(inputs) || (parts > 1 && mr.circuit_proofs[0] == mr.circuit_proofs[1])) {
            fprintf(stderr, "random-blinding proofs failed verification or repeated\n");
            return 2;
        }
        for (auto &p : mp.circuit_proofs) {
            for (uint8_t b : p) printf("%02x", b);
            printf("\n");
        }
        mi_synth_free(syn);
    } catch (const mi355x::error &e) {
        fprintf(stderr, "error %d: %s\n", e.code, e.what());
        return e.code == MI_ERR_NO_DEVICE ? 3 : 1;
    }
    return 0;
}
