// sdr.h -- SDR labelling witness (SHA-256 labels of challenged nodes), sdr.hip.  SURVEY.md §8(f)#3.
#pragma once
#include <cstdint>

namespace mi {
struct Ctx;

// replica_id as the eight big-endian SHA-256 message words of the first block
struct SdrReplica {
    uint32_t w[8];
};
SdrReplica sdr_replica(const uint8_t replica_id[32]);

// labels_out[i] (32 B) = create_label(replica_id, layers[i], nodes[i], parents[i * n_parents ..] repeated
// cyclically to 37); n_parents = 0: the parentless label of node 0
void sdr_labels_dev(Ctx &c, const SdrReplica &rid, const uint32_t *layers, const uint64_t *nodes,
                    const void *parents, uint32_t n_parents, uint64_t n, void *labels_out);
// the same with parents gathered from the device-resident layer labels (layer-major, layer l at entry
// (l - 1) * nodes_per_layer) by parent_idx[i * (n_base + n_exp) ..]; parents_out (optional) receives the 37
// repeated parent labels of each challenge
void sdr_labels_gather_dev(Ctx &c, const SdrReplica &rid, const void *layer_labels, uint64_t nodes_per_layer,
                           const uint32_t *layers, const uint64_t *challenges, const uint32_t *parent_idx,
                           uint32_t n_base, uint32_t n_exp, uint64_t n, void *labels_out, void *parents_out);
// tree D: every row above the leaves of the binary SHA-256 tree (node = SHA256(left || right), byte 31 &=
// 0x3f), bottom-up, n - 1 entries of 32 B; n a power of two
void tree_d_build_dev(Ctx &c, const void *leaves, uint64_t n, void *rows);
}  // namespace mi
