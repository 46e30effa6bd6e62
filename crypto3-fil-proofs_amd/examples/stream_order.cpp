// stream_order.cpp -- the stream-ordering contract of the device-pointer entries (include/mi355x_groth16.h,
// "device pointers") exercised the way a C++ caller of generate_tree_c_gpu / circuit_proofs would
// (porep/stacked/vanilla/proof.hpp:383-640, core/proof/compound_proof.hpp:127-137): inputs are produced and
// outputs cleared by hipMemcpyAsync / hipMemsetAsync on the caller's OWN non-blocking stream, behind a few
// milliseconds of unrelated work, and the library entries are called right after with no host
// synchronisation.  The library orders itself after that stream (context::set_caller_stream).
// Prints the tree C root and the proof (hex); tests/test_gpu_cpp.py compares them with the oracle.
//   stream_order <log8_nodes> [race]   ("race": name an idle stream instead -- the pre-contract behaviour, to
//                                       show what the rule prevents; its output is reported, never trusted)
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mi355x_groth16.hpp"

#define HIPCHK(x)                                                                      \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s line %d\n", #x, hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

static uint64_t splitmix(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static void hex32(const uint8_t *p) {
    for (int i = 31; i >= 0; i--) std::printf("%02x", p[i]);
    std::printf("\n");
}

int main(int argc, char **argv) {
    const int lg8 = argc > 1 ? std::atoi(argv[1]) : 3;
    const bool race = argc > 2 && std::strcmp(argv[2], "race") == 0;
    uint64_t nodes = 1;
    for (int i = 0; i < lg8; i++) nodes *= 8;
    try {
        mi355x::context ctx(0);
        hipStream_t prod, idle;
        HIPCHK(hipStreamCreateWithFlags(&prod, hipStreamNonBlocking));
        HIPCHK(hipStreamCreateWithFlags(&idle, hipStreamNonBlocking));
        ctx.set_caller_stream(race ? (void *)idle : (void *)prod);
        // unrelated work queued ahead on the producer stream, so a library that did not wait for the stream
        // would run before the inputs exist
        const size_t slow_bytes = 4ull << 30;
        void *slow = nullptr;
        HIPCHK(hipMalloc(&slow, slow_bytes));
        auto delay = [&] {
            for (int k = 0; k < 6; k++) HIPCHK(hipMemsetAsync(slow, k, slow_bytes, prod));
        };

        // ---- tree C (ColumnTreeBuilder::add_final_columns on device-resident labels) ----
        uint64_t seed = 42, tree_n = 0;
        mi355x::check(mi_tree_cache_size(nodes, 8, 0, &tree_n));
        uint8_t *labels_h = nullptr;
        HIPCHK(hipHostMalloc((void **)&labels_h, 32 * 11 * nodes, hipHostMallocDefault));
        for (uint64_t i = 0; i < 4 * 11 * nodes; i++) {  // layer-major, the same SplitMix64 stream as tree_c.cpp
            uint64_t w = splitmix(seed);
            if (i % 4 == 3) w &= 0x0FFFFFFFFFFFFFFFull;
            std::memcpy(labels_h + 8 * i, &w, 8);
        }
        void *labels_d, *base_d, *tree_d;
        HIPCHK(hipMalloc(&labels_d, 32 * 11 * nodes));
        HIPCHK(hipMalloc(&base_d, 32 * nodes));
        HIPCHK(hipMalloc(&tree_d, 32 * tree_n));
        delay();
        HIPCHK(hipMemcpyAsync(labels_d, labels_h, 32 * 11 * nodes, hipMemcpyHostToDevice, prod));
        HIPCHK(hipMemsetAsync(base_d, 0, 32 * nodes, prod));  // the caller clears its outputs
        HIPCHK(hipMemsetAsync(tree_d, 0, 32 * tree_n, prod));
        mi355x::check(mi_tree_c_build_dev(ctx.get(), 11, nodes, labels_d, 8, base_d, tree_d));
        uint8_t root[32];
        HIPCHK(hipMemcpyAsync(root, (uint8_t *)tree_d + 32 * (tree_n - 1), 32, hipMemcpyDeviceToHost, prod));
        HIPCHK(hipStreamSynchronize(prod));
        hex32(root);

        // ---- Groth16 over a device-resident witness (circuit_proofs with a GPU synthesiser upstream) ----
        mi_synth *syn = nullptr;
        mi355x::check(mi_synth_generate(10, 4, 1, &syn));
        mi_r1cs cs;
        mi355x::check(mi_synth_r1cs(syn, &cs));
        const uint8_t *zp = nullptr;
        uint64_t nv = 0;
        mi355x::check(mi_synth_witness(syn, &zp, &nv));
        mi355x::circuit circ(ctx, cs);
        std::array<mi355x::fr32, 5> toxic{};
        for (int i = 0; i < 5; i++) toxic[i][0] = (uint8_t)(11 + i);
        auto pk = mi355x::proving_key::generate(ctx, circ, toxic);
        uint8_t *z_h = nullptr;
        HIPCHK(hipHostMalloc((void **)&z_h, 32 * nv, hipHostMallocDefault));
        std::memcpy(z_h, zp, 32 * nv);
        void *z_d;
        HIPCHK(hipMalloc(&z_d, 32 * nv));
        HIPCHK(hipMemsetAsync(z_d, 0, 32 * nv, prod));
        HIPCHK(hipStreamSynchronize(prod));  // z_d starts as a valid all-zero witness
        delay();
        HIPCHK(hipMemcpyAsync(z_d, z_h, 32 * nv, hipMemcpyHostToDevice, prod));
        mi355x::fr32 r{}, s{};
        r[0] = 100;
        s[0] = 200;
        mi355x::proof_bytes proof = mi355x::prove_dev(ctx, pk, circ, z_d, r, s);
        for (uint8_t b : proof) std::printf("%02x", b);
        std::printf("\n");

        mi_synth_free(syn);
        HIPCHK(hipStreamSynchronize(prod));
        HIPCHK(hipFree(z_d));
        HIPCHK(hipHostFree(z_h));
        HIPCHK(hipFree(labels_d));
        HIPCHK(hipFree(base_d));
        HIPCHK(hipFree(tree_d));
        HIPCHK(hipHostFree(labels_h));
        HIPCHK(hipFree(slow));
        HIPCHK(hipStreamDestroy(prod));
        HIPCHK(hipStreamDestroy(idle));
    } catch (const mi355x::error &e) {
        std::fprintf(stderr, "error %d: %s\n", e.code, e.what());
        return e.code == MI_ERR_NO_DEVICE ? 3 : 1;
    }
    return 0;
}
