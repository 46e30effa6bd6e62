// mi355x_groth16.hpp -- header-only C++ host layer over the C ABI (mi355x_groth16.h).
//
// Mirrors the reference's prover-side C++ interface so a maintainer can swap the crypto3 CPU
// prover for the MI355X one behind the same call shapes:
//   * proving_key  ~ r1cs_gg_ppzksnark_mapped_scheme_params / scheme_params{vk,h,l,a,b_g1,b_g2}
//                    (libs/storage/include/nil/filecoin/storage/proofs/core/crypto/scheme_params.hpp:38-67)
//   * prove(...)   ~ crypto3 r1cs_gg_ppzksnark prove(pk, primary_input, auxiliary_input)
//   * circuit_proofs(...) ~ compound_proof::circuit_proofs partition loop (core/proof/compound_proof.hpp:127-137)
//   * multi_proof  ~ multi_proof{circuit_proofs, verifying_key} (core/proof/multi_proof.hpp:38-58),
//                    written as P x 192 bytes (api/seal.hpp:306-308)
//   * partition_count ~ core/partitions.hpp:36-38
//   * column_tree_builder / tree_builder / generate_tree_r_last / hash_single_column ~ the tree C / tree
//                    R-last builders and the column hash of porep/stacked/vanilla/proof.hpp:383-810 and
//                    porep/stacked/vanilla/hash.hpp:37-47
// Errors are thrown as mi355x::error, like the reference's BOOST_ASSERT_MSG / throw style
// (compound_proof.hpp:94).
#pragma once
#include <algorithm>
#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "mi355x_groth16.h"

namespace mi355x {

struct error : std::runtime_error {
    int code;
    error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

inline void check(int rc) {
    if (rc != MI_OK) throw error(rc, std::string("libfilgpu: ") + mi_last_error());
}

using fr32 = std::array<uint8_t, 32>;  // Fr, 32 bytes little-endian (core/fr32.hpp:36-52)
using proof_bytes = std::array<uint8_t, MI_PROOF_BYTES>;

inline std::int64_t partition_count(std::int64_t partitions) {  // core/partitions.hpp:36-38
    return partitions == -1 ? 1 : (partitions == 0 ? -1 : partitions);
}

class context {
public:
    explicit context(int device = 0) { check(mi_ctx_create(device, &h_)); }
    ~context() { mi_ctx_destroy(h_); }
    context(const context &) = delete;
    context &operator=(const context &) = delete;
    mi_ctx *get() const { return h_; }
    void synchronize() { check(mi_ctx_synchronize(h_)); }
    // The stream that produces this context's device inputs and consumes its device outputs (a hipStream_t;
    // nullptr = the legacy default stream).  Every entry taking a device pointer then waits, on the device,
    // for the work queued there before the call, and returns with its outputs written -- see "Device pointers"
    // in mi355x_groth16.h.  No host synchronisation is needed around the calls.
    void set_caller_stream(void *hip_stream) { check(mi_ctx_set_caller_stream(h_, hip_stream)); }

private:
    mi_ctx *h_ = nullptr;
};

class circuit {
public:
    circuit(context &ctx, const mi_r1cs &cs) { check(mi_circuit_load(ctx.get(), &cs, &h_)); }
    // a stacked-PoRep / Fallback-PoSt circuit built by the library, uploaded in its compact form
    circuit(context &ctx, const mi_stacked *built) { check(mi_stacked_load(ctx.get(), built, &h_)); }
    ~circuit() { mi_circuit_free(h_); }
    circuit(const circuit &) = delete;
    circuit &operator=(const circuit &) = delete;
    mi_circuit *get() const { return h_; }
    std::uint64_t num_variables() const {
        std::uint64_t info[9];
        check(mi_circuit_info(h_, info));
        return info[1] + info[2];
    }

private:
    mi_circuit *h_ = nullptr;
};

class proving_key {
public:
    // load a bellman-layout key (uncompressed points); checked -> on-curve validation
    proving_key(context &ctx, const circuit *c, const mi_srs_host &host, bool checked) {
        check(mi_srs_load(ctx.get(), c ? c->get() : nullptr, &host, checked ? 1 : 0, &h_));
    }
    // a bellman / filecoin v28-*.params file: mmapped and streamed to the device once
    // (read_cached_params / get_groth_params, core/parameter_cache.hpp:125-129,185-200)
    static proving_key from_params_file(context &ctx, const circuit *c, const std::string &path, bool checked) {
        mi_srs *h = nullptr;
        check(mi_params_load(ctx.get(), c ? c->get() : nullptr, path.c_str(), checked ? 1 : 0, &h));
        return proving_key(h);
    }
    void write_params(context &ctx, const std::string &path) const { check(mi_params_write(ctx.get(), h_, path.c_str())); }
    void write_vk(const std::string &path) const { check(mi_vk_write(h_, path.c_str())); }
    // groth16::generate_random_parameters with known toxic waste (tests / benches)
    static proving_key generate(context &ctx, const circuit &c, const std::array<fr32, 5> &toxic) {
        std::array<uint8_t, 160> t;
        for (int i = 0; i < 5; i++)
            for (int j = 0; j < 32; j++) t[32 * i + j] = toxic[i][j];
        mi_srs *h = nullptr;
        check(mi_srs_generate(ctx.get(), c.get(), t.data(), &h));
        return proving_key(h);
    }
    proving_key(proving_key &&o) noexcept : h_(std::exchange(o.h_, nullptr)) {}
    ~proving_key() { mi_srs_free(h_); }
    mi_srs *get() const { return h_; }
    std::vector<uint8_t> verifying_key() const {
        std::vector<uint8_t> vk(MI_VK_BYTES);
        check(mi_srs_export_vk(h_, vk.data(), nullptr));
        return vk;
    }
    std::vector<uint8_t> ic() const {
        uint64_t info[6];
        check(mi_srs_info(h_, info));
        std::vector<uint8_t> out(96 * info[5]);
        check(mi_srs_export_vk(h_, nullptr, out.data()));
        return out;
    }

private:
    explicit proving_key(mi_srs *h) : h_(h) {}
    mi_srs *h_ = nullptr;
};

// One proof: primary (ONE first) ++ auxiliary assignment, injected blinding r, s.
inline proof_bytes prove(context &ctx, const proving_key &pk, const circuit &c, const std::vector<fr32> &z,
                         const fr32 &r, const fr32 &s, bool priority = false) {
    if (z.size() != c.num_variables()) throw error(MI_ERR_ARG, "assignment length != number of variables");
    proof_bytes out;
    check(mi_groth16_prove(ctx.get(), pk.get(), c.get(), z.front().data(), r.data(), s.data(), priority ? 1 : 0,
                           out.data(), nullptr));
    return out;
}

// The production call: r, s drawn inside the library from getrandom() (crypto3 prove / bellman
// create_random_proof); the overload above with injected r, s is the parity/test entry.
inline proof_bytes prove(context &ctx, const proving_key &pk, const circuit &c, const std::vector<fr32> &z,
                         bool priority = false) {
    if (z.size() != c.num_variables()) throw error(MI_ERR_ARG, "assignment length != number of variables");
    proof_bytes out;
    check(mi_groth16_prove_random(ctx.get(), pk.get(), c.get(), z.front().data(), priority ? 1 : 0, out.data()));
    return out;
}

// A witness already in device memory (a GPU synthesiser's output, e.g. mi_stacked_witness_dev): the call waits on
// the device for the work queued on the context's caller stream before it (context::set_caller_stream), so the
// producer's kernels and copies need no host synchronisation in between.
inline proof_bytes prove_dev(context &ctx, const proving_key &pk, const circuit &c, const void *z_dev, const fr32 &r,
                             const fr32 &s, bool priority = false) {
    proof_bytes out;
    check(mi_groth16_prove_dev(ctx.get(), pk.get(), c.get(), z_dev, r.data(), s.data(), priority ? 1 : 0, out.data(),
                               nullptr));
    return out;
}

// bellman verify_proof on the host; inputs = public inputs without ONE (generate_public_inputs order)
inline bool verify(const std::vector<uint8_t> &vk, const std::vector<uint8_t> &ic, const std::vector<fr32> &inputs,
                   const proof_bytes &proof) {
    if (ic.size() / 96 != inputs.size() + 1) throw error(MI_ERR_ARG, "inputs.size() must be |ic| - 1");
    int ok = 0;
    check(mi_groth16_verify(vk.data(), ic.data(), ic.size() / 96, inputs.empty() ? nullptr : inputs.front().data(),
                            proof.data(), &ok));
    return ok != 0;
}

struct multi_proof {
    std::vector<proof_bytes> circuit_proofs;
    std::vector<uint8_t> verifying_key;
    std::vector<uint8_t> ic;
    // verify_seal's batch check over all partitions (api/seal.hpp:339-485); weights from getrandom(),
    // or from the ChaCha20 stream of seed32 (32 B, tests only) when given
    bool verify(const std::vector<std::vector<fr32>> &public_inputs, const uint8_t *seed32 = nullptr) const {
        if (public_inputs.size() != circuit_proofs.size()) throw error(MI_ERR_ARG, "one input vector per partition");
        std::vector<uint8_t> in, pr;
        for (auto &v : public_inputs) {
            if (v.size() + 1 != ic.size() / 96) throw error(MI_ERR_ARG, "inputs.size() must be |ic| - 1");
            for (auto &x : v) in.insert(in.end(), x.begin(), x.end());
        }
        for (auto &p : circuit_proofs) pr.insert(pr.end(), p.begin(), p.end());
        int ok = 0;
        const uint8_t *ins = in.empty() ? nullptr : in.data(), *prs = pr.empty() ? nullptr : pr.data();
        if (seed32)
            check(mi_groth16_verify_batch_seeded(verifying_key.data(), ic.data(), ic.size() / 96,
                                                 circuit_proofs.size(), ins, prs, seed32, &ok));
        else
            check(mi_groth16_verify_batch(verifying_key.data(), ic.data(), ic.size() / 96, circuit_proofs.size(),
                                          ins, prs, &ok));
        return ok != 0;
    }
    std::vector<uint8_t> write() const {  // api/seal.hpp:306-308
        std::vector<uint8_t> buf;
        buf.reserve(circuit_proofs.size() * MI_PROOF_BYTES);
        for (auto &p : circuit_proofs) buf.insert(buf.end(), p.begin(), p.end());
        return buf;
    }
};

namespace detail {
inline multi_proof circuit_proofs_impl(context &ctx, const proving_key &pk, const circuit &c,
                                       const std::vector<std::vector<fr32>> &partition_assignments,
                                       const std::vector<std::pair<fr32, fr32>> *blindings, bool priority) {
    if (partition_assignments.empty())
        throw error(MI_ERR_ARG, "Cannot create a circuit proof over missing vanilla proofs");
    if (blindings && blindings->size() != partition_assignments.size())
        throw error(MI_ERR_ARG, "one (r, s) per partition");
    std::vector<const uint8_t *> zs;
    for (auto &z : partition_assignments) {
        if (z.size() != c.num_variables()) throw error(MI_ERR_ARG, "assignment length != number of variables");
        zs.push_back(z.front().data());
    }
    std::vector<uint8_t> out(MI_PROOF_BYTES * zs.size());
    if (blindings) {
        std::vector<uint8_t> rs;
        for (auto &b : *blindings) {
            rs.insert(rs.end(), b.first.begin(), b.first.end());
            rs.insert(rs.end(), b.second.begin(), b.second.end());
        }
        check(mi_groth16_prove_batch(ctx.get(), pk.get(), c.get(), zs.size(), zs.data(), rs.data(), priority ? 1 : 0,
                                     out.data()));
    } else {
        check(mi_groth16_prove_batch_random(ctx.get(), pk.get(), c.get(), zs.size(), zs.data(), priority ? 1 : 0,
                                            out.data()));
    }
    multi_proof mp;
    for (size_t k = 0; k < zs.size(); k++) {
        proof_bytes p;
        std::copy(out.begin() + MI_PROOF_BYTES * k, out.begin() + MI_PROOF_BYTES * (k + 1), p.begin());
        mp.circuit_proofs.push_back(p);
    }
    mp.verifying_key = pk.verifying_key();
    mp.ic = pk.ic();
    return mp;
}
}  // namespace detail

// compound_proof::circuit_proofs (compound_proof.hpp:127-137): one Groth16 proof per partition, in partition
// order, through mi_groth16_prove_batch (partition k + 1's witness upload and proof k's host assembly overlap
// proof k's GPU work).  Production form: r, s drawn inside the library for every partition.
inline multi_proof circuit_proofs(context &ctx, const proving_key &pk, const circuit &c,
                                  const std::vector<std::vector<fr32>> &partition_assignments, bool priority = false) {
    return detail::circuit_proofs_impl(ctx, pk, c, partition_assignments, nullptr, priority);
}
// parity/test form with injected (r, s) per partition
inline multi_proof circuit_proofs(context &ctx, const proving_key &pk, const circuit &c,
                                  const std::vector<std::vector<fr32>> &partition_assignments,
                                  const std::vector<std::pair<fr32, fr32>> &blindings, bool priority = false) {
    return detail::circuit_proofs_impl(ctx, pk, c, partition_assignments, &blindings, priority);
}

// ---- stacked-PoRep Poseidon trees ----------------------------------------------
// Fr values are 32-byte little-endian canonical (< r); trees are returned row by row, bottom-up, without
// the base row (and without the rows_to_discard lowest rows above it).
inline std::uint64_t merkle_tree_cache_size(std::uint64_t leafs, unsigned arity, unsigned rows_to_discard) {
    std::uint64_t n = 0;
    check(mi_tree_cache_size(leafs, arity, rows_to_discard, &n));  // get_merkle_tree_cache_size
    return n;
}

// hash_single_column (porep/stacked/vanilla/hash.hpp:37-47): Poseidon over 2 or 11 labels
inline fr32 hash_single_column(context &ctx, const std::vector<fr32> &column) {
    if (column.size() != 2 && column.size() != 11) throw error(MI_ERR_ARG, "unsupported column size");
    fr32 out{};
    check(mi_poseidon_hash(ctx.get(), (unsigned)column.size(), column.front().data(), 1, out.data()));
    return out;
}

// ColumnTreeBuilder<ColumnArity, TreeArity>::add_final_columns -> (base_data, tree_data)
class column_tree_builder {
public:
    column_tree_builder(context &ctx, unsigned column_arity = 11, unsigned tree_arity = 8)
        : ctx_(ctx), column_arity_(column_arity), tree_arity_(tree_arity) {}
    // layers[l] points at the nodes labels of layer l + 1 for this sub-tree (32 B each)
    std::pair<std::vector<uint8_t>, std::vector<uint8_t>> add_final_columns(const std::vector<const uint8_t *> &layers,
                                                                            std::uint64_t nodes) const {
        if (layers.size() != column_arity_) throw error(MI_ERR_ARG, "one label vector per column layer");
        std::vector<uint8_t> base(32 * nodes), tree(32 * merkle_tree_cache_size(nodes, tree_arity_, 0));
        check(mi_tree_c_build(ctx_.get(), column_arity_, nodes, layers.data(), tree_arity_, base.data(), tree.data()));
        return {std::move(base), std::move(tree)};
    }

private:
    context &ctx_;
    unsigned column_arity_, tree_arity_;
};

// TreeBuilder<Arity>::add_final_leaves -> tree_data
class tree_builder {
public:
    tree_builder(context &ctx, unsigned arity = 8, unsigned rows_to_discard = 0)
        : ctx_(ctx), arity_(arity), rows_to_discard_(rows_to_discard) {}
    std::vector<uint8_t> add_final_leaves(const uint8_t *leaves, std::uint64_t n) const {
        std::vector<uint8_t> tree(32 * merkle_tree_cache_size(n, arity_, rows_to_discard_));
        check(mi_tree_build(ctx_.get(), arity_, leaves, n, rows_to_discard_, tree.data()));
        return tree;
    }

private:
    context &ctx_;
    unsigned arity_, rows_to_discard_;
};

// generate_tree_r_last, GPU branch: data (the sector's nodes) becomes the replica in place
// (encode: label + data), then the tree over it
inline std::vector<uint8_t> generate_tree_r_last(context &ctx, std::uint64_t nodes, const uint8_t *last_layer_labels,
                                                 uint8_t *data, unsigned arity = 8, unsigned rows_to_discard = 0) {
    std::vector<uint8_t> tree(32 * merkle_tree_cache_size(nodes, arity, rows_to_discard));
    check(mi_tree_r_last_build(ctx.get(), nodes, last_layer_labels, data, arity, rows_to_discard, tree.data()));
    return tree;
}

// ---- SDR labelling witness ----
// labels[i] = create_label(replica_id, layers[i], nodes[i], n_parents parents of entry i repeated to 37)
inline std::vector<fr32> create_labels(context &ctx, const fr32 &replica_id, const std::vector<std::uint32_t> &layers,
                                       const std::vector<std::uint64_t> &nodes, const std::vector<fr32> &parents,
                                       unsigned n_parents) {
    if (layers.size() != nodes.size() || parents.size() != (size_t)n_parents * layers.size())
        throw error(MI_ERR_ARG, "create_labels: layers, nodes and parents disagree");
    std::vector<fr32> out(layers.size());
    if (!layers.empty())
        check(mi_sdr_labels(ctx.get(), replica_id.data(), layers.size(), layers.data(), nodes.data(),
                            n_parents ? parents.front().data() : nullptr, n_parents, out.front().data()));
    return out;
}

// LabelingProof (porep/stacked/vanilla/labelling_proof.hpp:40-48) with create_label / verify as in
// vanilla/detail/processing/naive/labelling_proof.hpp:46-70; EncodingProof::create_key is the same hash
struct labeling_proof {
    std::vector<fr32> parents;  // parents_data_full (37), or the distinct parents (repeated to 37)
    std::uint32_t layer_index = 0;
    std::uint64_t node = 0;

    fr32 create_label(context &ctx, const fr32 &replica_id) const {
        return create_labels(ctx, replica_id, {layer_index}, {node}, parents, (unsigned)parents.size()).front();
    }
    bool verify(context &ctx, const fr32 &replica_id, const fr32 &expected_label) const {
        return create_label(ctx, replica_id) == expected_label;
    }
};

}  // namespace mi355x
