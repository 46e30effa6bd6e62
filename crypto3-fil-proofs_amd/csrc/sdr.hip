// sdr.hip -- SDR labelling witness of stacked PoRep on CDNA4 (gfx950).  SURVEY.md §8(f)#3.
//
// The labelling and encoding proofs of every challenge carry the label of the challenged node, recomputed
// from its 37 parent labels (vanilla/proof.hpp:196-255 builds parents_data_full, LabelingProof::create_label
// hashes it: vanilla/detail/processing/naive/labelling_proof.hpp:46-60; EncodingProof::create_key is the same
// hash: vanilla/encoding_proof.hpp:42-53).  The message is
//   replica_id (32) || u32_be(layer) || u64_be(node) || 0^20 || parent[0] .. parent[36] (32 each),
// SHA-256 over 1248 bytes = 20 compression blocks (the last one carries parent 36 and the padding), then
// byte 31 &= 0x3f (create_label.hpp:76-77).  Parents are the node's base parents (current layer) and, from
// layer 2 on, its expander parents (previous layer), repeated cyclically to 37 (proof.hpp:233-237).
// Node 0 has no parents: its label hashes the 64-byte prefix alone (create_label.hpp:67-69).
//
// Device form: one thread per label, all of SHA-256 in 32-bit VALU registers (rotations are
// v_alignbit_b32, Ch / Maj are v_bfi_b32, the sums v_add3_u32); the 64 rounds of one compression are
// unrolled over a rolling 16-word schedule window and the block loop is not (≈ 1.5 K instructions of
// code, resident in the instruction cache).  The kernel is VALU-bound: ≈ 29 K lane-ops per label against
// ≈ 1.2 KB of parent bytes, so parents are read straight from HBM (two 16-byte loads per parent) with no
// LDS staging.  Two input forms:
//   * k_sdr_labels: parent labels given per entry (n_parents per label, 0..37), the LabelingProof layout;
//   * k_sdr_labels_gather: parents gathered from the device-resident layer labels by node index
//     (base parents from the challenged layer, expander parents from the layer below), optionally writing
//     the 37 repeated parent labels out as the proof's parents_data_full.
#include <cstdlib>

#include "ctx.h"
#include "sdr.h"

namespace mi {

namespace {

__constant__ uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

constexpr uint32_t kTotalParents = 37;                       // vanilla/proof.hpp:49
constexpr uint32_t kMsgBits = (64 + kTotalParents * 32) * 8;  // 9984

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
// x ^ y ^ z as one v_bitop3_b32 (truth table 0x96); left to itself the compiler emits two v_xor_b32
__device__ __forceinline__ uint32_t xor3(uint32_t x, uint32_t y, uint32_t z) {
    return __builtin_amdgcn_bitop3_b32(x, y, z, 0x96);
}

// K values are compile-time indices into a __constant__ table: with the rounds unrolled they become
// scalar loads (wave-uniform), not VALU work
__device__ __forceinline__ void compress(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int t = 0; t < 64; t++) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
            w[t & 15] = wt;
        }
        const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        const uint32_t ch = (e & f) ^ (~e & g);
        const uint32_t t1 = (h + kK[t] + wt) + S1 + ch;  // h + K + W is off the e -> e chain
        const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        const uint32_t maj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);  // majority (symmetric table)
        h = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + S0 + maj;
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
    st[4] += e;
    st[5] += f;
    st[6] += g;
    st[7] += h;
}

__device__ __forceinline__ void load_parent(const uint4 *__restrict__ p, uint32_t *w) {
    const uint4 lo = p[0], hi = p[1];
    w[0] = __builtin_bswap32(lo.x);
    w[1] = __builtin_bswap32(lo.y);
    w[2] = __builtin_bswap32(lo.z);
    w[3] = __builtin_bswap32(lo.w);
    w[4] = __builtin_bswap32(hi.x);
    w[5] = __builtin_bswap32(hi.y);
    w[6] = __builtin_bswap32(hi.z);
    w[7] = __builtin_bswap32(hi.w);
}

// label of one node given a parent-fetch functor fetch(k, w8) for k in [0, 37) (already cyclic)
template <class Fetch>
__device__ __forceinline__ void label_one(const SdrReplica &rid, uint32_t layer, uint64_t node, bool has_parents,
                                          Fetch &&fetch, uint4 *__restrict__ out) {
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = rid.w[j];
    w[8] = layer;
    w[9] = (uint32_t)(node >> 32);
    w[10] = (uint32_t)node;
#pragma unroll
    for (int j = 11; j < 16; j++) w[j] = 0;
    compress(st, w);
    uint32_t bits = 512;
    if (has_parents) {
#pragma unroll 1
        for (uint32_t k = 0; k < kTotalParents - 1; k += 2) {
            fetch(k, w);
            fetch(k + 1, w + 8);
            compress(st, w);
        }
        fetch(kTotalParents - 1, w);
        bits = kMsgBits;
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) w[j] = 0;
    }
    // padding block: 0x80 after the message, length in bits at the end (the message ends on a 32-byte
    // boundary: parent 36 in words 0-7, or nothing after the 64-byte prefix)
#pragma unroll
    for (int j = 8; j < 16; j++) w[j] = 0;
    if (has_parents) w[8] = 0x80000000u;
    else w[0] = 0x80000000u;
    w[15] = bits;
    compress(st, w);
    st[7] &= 0xffffff3fu;  // byte 31 (the last byte of the big-endian digest) &= 0x3f
    out[0] = make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]), __builtin_bswap32(st[2]),
                        __builtin_bswap32(st[3]));
    out[1] = make_uint4(__builtin_bswap32(st[4]), __builtin_bswap32(st[5]), __builtin_bswap32(st[6]),
                        __builtin_bswap32(st[7]));
}

__device__ __forceinline__ void unpack_parent(const uint4 *raw, uint32_t *w) {
    const uint4 lo = raw[0], hi = raw[1];
    w[0] = __builtin_bswap32(lo.x);
    w[1] = __builtin_bswap32(lo.y);
    w[2] = __builtin_bswap32(lo.z);
    w[3] = __builtin_bswap32(lo.w);
    w[4] = __builtin_bswap32(hi.x);
    w[5] = __builtin_bswap32(hi.y);
    w[6] = __builtin_bswap32(hi.z);
    w[7] = __builtin_bswap32(hi.w);
}

// software-pipelined form of label_one: the next block's two parents are loaded (raw, 4 x 16 B) before the
// current block is compressed, so a wave's own gather latency overlaps its hashing.  fetch_raw(k, raw2)
// issues the loads of parent k; sink(k, raw2) sees parent k when it is consumed (parents_data_full stores).
template <class FetchRaw, class Sink>
__device__ __forceinline__ void label_one_pf(const SdrReplica &rid, uint32_t layer, uint64_t node, bool has_parents,
                                             FetchRaw &&fetch_raw, Sink &&sink, uint4 *__restrict__ out) {
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = rid.w[j];
    w[8] = layer;
    w[9] = (uint32_t)(node >> 32);
    w[10] = (uint32_t)node;
#pragma unroll
    for (int j = 11; j < 16; j++) w[j] = 0;
    uint4 nx[4];
    if (has_parents) {
        fetch_raw(0, nx);
        fetch_raw(1, nx + 2);
    }
    compress(st, w);  // the prefix block overlaps the first gathers
    uint32_t bits = 512;
    if (has_parents) {
#pragma unroll 1
        for (uint32_t k = 0; k < kTotalParents - 1; k += 2) {
            sink(k, nx);
            sink(k + 1, nx + 2);
            unpack_parent(nx, w);
            unpack_parent(nx + 2, w + 8);
            if (k + 2 < kTotalParents - 1) {
                fetch_raw(k + 2, nx);
                fetch_raw(k + 3, nx + 2);
            } else {
                fetch_raw(kTotalParents - 1, nx);
            }
            compress(st, w);
        }
        sink(kTotalParents - 1, nx);
        unpack_parent(nx, w);
        bits = kMsgBits;
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) w[j] = 0;
    }
#pragma unroll
    for (int j = 8; j < 16; j++) w[j] = 0;
    if (has_parents) w[8] = 0x80000000u;
    else w[0] = 0x80000000u;
    w[15] = bits;
    compress(st, w);
    st[7] &= 0xffffff3fu;
    out[0] = make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]), __builtin_bswap32(st[2]),
                        __builtin_bswap32(st[3]));
    out[1] = make_uint4(__builtin_bswap32(st[4]), __builtin_bswap32(st[5]), __builtin_bswap32(st[6]),
                        __builtin_bswap32(st[7]));
}

__global__ void __launch_bounds__(256) k_sdr_labels(SdrReplica rid, const uint32_t *__restrict__ layers,
                                                    const uint64_t *__restrict__ nodes,
                                                    const uint4 *__restrict__ parents, uint32_t np, uint64_t n,
                                                    uint4 *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 *p = parents + i * np * 2;
    uint32_t cur = 0;  // parent index mod np, advanced in fetch order (k = 0, 1, .., 36)
    auto fetch = [&](uint32_t, uint32_t *w) __attribute__((always_inline)) {
        load_parent(p + 2 * cur, w);
        cur = cur + 1 == np ? 0 : cur + 1;
    };
    label_one(rid, layers[i], nodes[i], np != 0, fetch, out + 2 * i);
}

// parents gathered from the device-resident layers: labels_dev is layer-major (layer l, 1-based, at entry
// (l - 1) * nodes_per_layer).  parent_idx holds n_base + n_exp node indices per challenge; at layer 1 only
// the n_base base parents take part (proof.hpp:196-209), at layer >= 2 base parents read layer l and
// expander parents layer l - 1 (proof.hpp:210-231).  full_out (optional) receives the 37 repeated parent
// labels per challenge (LabelingProof::parents).
template <bool PF>
__global__ void __launch_bounds__(256) k_sdr_labels_gather(SdrReplica rid, const uint4 *__restrict__ labels,
                                                           uint64_t nodes_per_layer,
                                                           const uint32_t *__restrict__ layers,
                                                           const uint64_t *__restrict__ challenges,
                                                           const uint32_t *__restrict__ parent_idx,
                                                           uint32_t n_base, uint32_t n_exp, uint64_t n,
                                                           uint4 *__restrict__ out, uint4 *__restrict__ full_out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t layer = layers[i];
    const uint32_t np = layer == 1 ? n_base : n_base + n_exp;
    const uint32_t *pi = parent_idx + i * (uint64_t)(n_base + n_exp);
    const uint4 *cur_layer = labels + (uint64_t)(layer - 1) * nodes_per_layer * 2;
    const uint4 *prev_layer = layer >= 2 ? labels + (uint64_t)(layer - 2) * nodes_per_layer * 2 : cur_layer;
    uint4 *fo = full_out ? full_out + i * kTotalParents * 2 : nullptr;
    uint32_t cur = 0;
    auto fetch = [&](uint32_t k, uint32_t *w) __attribute__((always_inline)) {
        const uint32_t node = pi[cur];
        const uint4 *src = (cur < n_base ? cur_layer : prev_layer) + (uint64_t)node * 2;
        if (fo) {
            fo[2 * k] = src[0];
            fo[2 * k + 1] = src[1];
        }
        load_parent(src, w);
        cur = cur + 1 == np ? 0 : cur + 1;
    };
    const bool has = np != 0 && challenges[i] != 0;
    if constexpr (PF) {
        uint32_t nxt = 0;
        auto fetch_raw = [&](uint32_t, uint4 *raw) __attribute__((always_inline)) {
            const uint32_t node = pi[nxt];
            const uint4 *src = (nxt < n_base ? cur_layer : prev_layer) + (uint64_t)node * 2;
            raw[0] = src[0];
            raw[1] = src[1];
            nxt = nxt + 1 == np ? 0 : nxt + 1;
        };
        auto sink = [&](uint32_t k, const uint4 *raw) __attribute__((always_inline)) {
            if (fo) {
                fo[2 * k] = raw[0];
                fo[2 * k + 1] = raw[1];
            }
        };
        label_one_pf(rid, layer, challenges[i], has, fetch_raw, sink, out + 2 * i);
    } else {
        label_one(rid, layer, challenges[i], has, fetch, out + 2 * i);
    }
}

// tree D (the SHA-256 binary tree over the sector's data, comm_d; openings at vanilla/proof.hpp:139-140):
// out[i] = SHA256(in[2i] || in[2i + 1]) with byte 31 &= 0x3f (Sha256Hasher's node hash, truncated into Fr).
// Two compressions per node: the 64-byte message block, then the constant padding block (length 512).
__global__ void __launch_bounds__(256) k_sha256_pairs(const uint4 *__restrict__ in, uint64_t n_out,
                                                      uint4 *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_out) return;
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint32_t w[16];
    load_parent(in + 4 * i, w);
    load_parent(in + 4 * i + 2, w + 8);
    compress(st, w);
    w[0] = 0x80000000u;
#pragma unroll
    for (int j = 1; j < 15; j++) w[j] = 0;
    w[15] = 512;
    compress(st, w);
    st[7] &= 0xffffff3fu;
    out[2 * i] = make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]), __builtin_bswap32(st[2]),
                            __builtin_bswap32(st[3]));
    out[2 * i + 1] = make_uint4(__builtin_bswap32(st[4]), __builtin_bswap32(st[5]), __builtin_bswap32(st[6]),
                                __builtin_bswap32(st[7]));
}

inline unsigned grid256(uint64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

SdrReplica sdr_replica(const uint8_t replica_id[32]) {
    SdrReplica r;
    for (int j = 0; j < 8; j++)
        r.w[j] = (uint32_t)replica_id[4 * j] << 24 | (uint32_t)replica_id[4 * j + 1] << 16 |
                 (uint32_t)replica_id[4 * j + 2] << 8 | replica_id[4 * j + 3];
    return r;
}

void sdr_labels_dev(Ctx &c, const SdrReplica &rid, const uint32_t *layers, const uint64_t *nodes,
                    const void *parents, uint32_t n_parents, uint64_t n, void *labels_out) {
    if (!n) return;
    if (n_parents > kTotalParents) throw std::invalid_argument("sdr: n_parents must be <= 37");
    k_sdr_labels<<<grid256(n), 256, 0, c.stream>>>(rid, layers, nodes, (const uint4 *)parents, n_parents, n,
                                                   (uint4 *)labels_out);
    MI_LAUNCHED(c, "k_sdr_labels");
}

void sdr_labels_gather_dev(Ctx &c, const SdrReplica &rid, const void *layer_labels, uint64_t nodes_per_layer,
                           const uint32_t *layers, const uint64_t *challenges, const uint32_t *parent_idx,
                           uint32_t n_base, uint32_t n_exp, uint64_t n, void *labels_out, void *parents_out) {
    if (!n) return;
    if (n_base + n_exp > kTotalParents || n_base == 0)
        throw std::invalid_argument("sdr: 1 <= n_base and n_base + n_exp <= 37");
    // tune::SDR_PREFETCH (A/B, tests): 1 = software-pipelined parent gathers, 0 = load at use
    const bool pf = tune::get(tune::SDR_PREFETCH, 0) != 0;
    if (pf)
        k_sdr_labels_gather<true><<<grid256(n), 256, 0, c.stream>>>(rid, (const uint4 *)layer_labels,
                                                                    nodes_per_layer, layers, challenges, parent_idx,
                                                                    n_base, n_exp, n, (uint4 *)labels_out,
                                                                    (uint4 *)parents_out);
    else
        k_sdr_labels_gather<false><<<grid256(n), 256, 0, c.stream>>>(rid, (const uint4 *)layer_labels,
                                                                     nodes_per_layer, layers, challenges, parent_idx,
                                                                     n_base, n_exp, n, (uint4 *)labels_out,
                                                                     (uint4 *)parents_out);
    MI_LAUNCHED(c, "k_sdr_labels_gather");
}

void tree_d_build_dev(Ctx &c, const void *leaves, uint64_t n, void *rows) {
    if (n < 2 || (n & (n - 1))) throw std::invalid_argument("tree D: the leaf count must be a power of two >= 2");
    const uint4 *cur = (const uint4 *)leaves;
    uint4 *dst = (uint4 *)rows;
    for (uint64_t m = n / 2; m >= 1; m /= 2) {
        k_sha256_pairs<<<grid256(m), 256, 0, c.stream>>>(cur, m, dst);
        MI_LAUNCHED(c, "k_sha256_pairs");
        cur = dst;
        dst += 2 * m;
    }
}

}  // namespace mi
