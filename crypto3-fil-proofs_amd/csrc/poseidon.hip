// poseidon.hip -- Poseidon over the BLS12-381 scalar field and the Poseidon Merkle-tree builders of
// stacked PoRep (tree C, tree R-last) for CDNA4 (gfx950).  SURVEY.md §8(f)#4.
//
// Reference: the column hash `hash_single_column` calls crypto3's poseidon<FieldType, 11, 11> / <.., 2, 2>
// (libs/storage/include/nil/filecoin/storage/proofs/porep/stacked/vanilla/hash.hpp:37-47); tree C is
// ColumnTreeBuilder<ColumnArity, TreeArity>::add_final_columns (column hashes, then an arity-8 Poseidon
// tree over them) and tree R-last is TreeBuilder<8>::add_final_leaves over the encoded replica
// (porep/stacked/vanilla/proof.hpp:383-810; GPU switches at core/configuration.hpp:51-56).  The hash
// itself lives in the empty crypto3 hash submodule, so the construction is restated from Filecoin's
// published parameters (oracle/poseidon_ref.py states every choice; parity unpinned):
//   state = [2^arity - 1, x_1 .. x_arity], x^5 S-box, R_F = 8 full and R_P partial rounds, Cauchy MDS
//   M[i][j] = 1 / (i + j + t), Grain-LFSR round constants, digest = state[1].
//
// Device evaluation (same permutation, cheaper form):
//   * Fr lives in 9 x 29-bit limbs (Montgomery R = 2^261, the radix of fr_t) for the whole permutation,
//     values lazily in [0, 4r): a product of operands below ~64r is < 2r (REDC bound, r / R < 2^-6), and
//     a column of <= 63 products < 2^58 fits one 64-bit accumulator, so an MDS row of up to 6 terms is
//     ONE product-scanning pass with a single Montgomery reduction (K multiplications, 1 reduction).
//   * Partial rounds use the sparse factorisation of M: the round constants of elements 1.. are folded
//     forward into the next round, and M A_{k-1} = A_k B_k with A_k = diag(1, M^_k) block-diagonal and
//     B_k = [[m00, v^T A^_{k-1}], [A^_k^-1 w, I]] sparse (2t - 1 multiplications instead of t^2); the last
//     partial round applies the dense M A_{R_P - 1}.  All of it is derived on the host at first use.
//   * Round constants and matrices are wave-uniform: they are read with scalar loads.
//   * One thread per hash; tree levels are launched bottom-up on the device, columns are read
//     layer-major (coalesced across threads).
#include <map>
#include <memory>
#include <utility>

#include "ctx.h"
#include "poseidon.h"
#include "poseidon_math.h"

namespace mi {

// out[i] = Poseidon(tag, x_{i,0} .. x_{i,A-1}), x_{i,j} = in[i * stride_hash + j * stride_elem]
// (canonical little-endian Fr, as stored); out canonical.
template <int T>
__global__ void __launch_bounds__(256) k_poseidon(const fr_t *__restrict__ in, uint64_t n, uint64_t stride_hash,
                                                  uint64_t stride_elem, PosK k, fr_t *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const fr29_t r2 = k.img[k.off_tag + 1];
    fr29_t s[T];
    s[0] = k.img[k.off_tag];
    const fr_t *p = in + i * stride_hash;
    sfor<T - 1>([&](auto j) { s[j + 1] = fr29_mul(fr29_from_fr(p[(uint64_t)j * stride_elem]), r2); });
    out[i] = fr_from_fr29(fr29_from_mont(poseidon_permute<T>(s, k)));
}

// replica = label + data (mod r), written back over data: the tree R-last leaves (porep encode)
__global__ void k_encode(const fr_t *__restrict__ key, fr_t *__restrict__ data, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    data[i] = key[i] + data[i];  // canonical operands < r: the sum reduced once is canonical
}

namespace {
inline unsigned grid256(uint64_t n) { return (unsigned)((n + 255) / 256); }

struct PosCache {
    std::map<unsigned, std::pair<PoseidonHost, fr29_t *>> m;
    ~PosCache() {
        for (auto &kv : m)
            if (kv.second.second) hipFree(kv.second.second);
    }
};
std::mutex g_pos_mu;
std::map<Ctx *, std::unique_ptr<PosCache>> g_pos;
}  // namespace

const PoseidonHost &poseidon_tables(Ctx &c, unsigned arity, PosK *dev) {
    std::lock_guard<std::mutex> g(g_pos_mu);
    auto &pc = g_pos[&c];
    if (!pc) pc.reset(new PosCache());
    const unsigned key = arity | poseidon_sbox_field() << 8;
    auto it = pc->m.find(key);
    if (it == pc->m.end()) {
        PoseidonHost h = poseidon_derive(arity, poseidon_sbox_field());
        fr29_t *d = nullptr;
        MI_HIP(hipMalloc(&d, h.img.size() * sizeof(fr29_t)));
        MI_HIP(hipMemcpy(d, h.img.data(), h.img.size() * sizeof(fr29_t), hipMemcpyHostToDevice));
        it = pc->m.emplace(key, std::make_pair(std::move(h), d)).first;
    }
    if (dev) {
        const PoseidonHost &h = it->second.first;
        *dev = PosK{it->second.second, (int)h.rf, (int)h.rp, (uint32_t)h.off_tag, (uint32_t)h.off_rc_first,
                    (uint32_t)h.off_rc_part, (uint32_t)h.off_rc_last, (uint32_t)h.off_mds, (uint32_t)h.off_sparse,
                    (uint32_t)h.off_dense};
    }
    return it->second.first;
}

void poseidon_free(Ctx &c) {
    std::lock_guard<std::mutex> g(g_pos_mu);
    g_pos.erase(&c);
}

void poseidon_hash_dev(Ctx &c, unsigned arity, const fr_t *in, uint64_t n, uint64_t stride_hash,
                       uint64_t stride_elem, fr_t *out) {
    if (!n) return;
    PosK k;
    poseidon_tables(c, arity, &k);
    ScopedTimer tm(c, &c.stats.poseidon, n);
    switch (arity) {
        case 2: k_poseidon<3><<<grid256(n), 256, 0, c.stream>>>(in, n, stride_hash, stride_elem, k, out); break;
        case 4: k_poseidon<5><<<grid256(n), 256, 0, c.stream>>>(in, n, stride_hash, stride_elem, k, out); break;
        case 8: k_poseidon<9><<<grid256(n), 256, 0, c.stream>>>(in, n, stride_hash, stride_elem, k, out); break;
        case 11: k_poseidon<12><<<grid256(n), 256, 0, c.stream>>>(in, n, stride_hash, stride_elem, k, out); break;
        default: throw std::invalid_argument("poseidon: arity must be 2, 4, 8 or 11");
    }
    MI_LAUNCHED(c, "k_poseidon");
}

void encode_dev(Ctx &c, const fr_t *key, fr_t *data, uint64_t n) {
    if (!n) return;
    k_encode<<<grid256(n), 256, 0, c.stream>>>(key, data, n);
    MI_LAUNCHED(c, "k_encode");
}

uint64_t tree_rows_size(uint64_t leaves, unsigned arity, unsigned rows_to_discard) {
    // every row above the base except the rows_to_discard lowest of them (merkletree
    // get_merkle_tree_cache_size; rows_to_discard = 0: the whole tree minus the base)
    if (arity < 2 || leaves == 0) throw std::invalid_argument("tree: arity >= 2 and at least one leaf");
    uint64_t size = 0, row = leaves;
    unsigned level = 0;
    while (row > 1) {
        if (row % arity) throw std::invalid_argument("tree: leaf count is not a power of the arity");
        row /= arity;
        level++;
        if (level > rows_to_discard) size += row;
    }
    if (rows_to_discard >= level && level > 0) throw std::invalid_argument("tree: cannot discard every row but the root");
    return size;
}

void tree_build_dev(Ctx &c, unsigned arity, const fr_t *leaves, uint64_t n, unsigned rows_to_discard, fr_t *rows,
                    fr_t *discard_tmp) {
    // rows: tree_rows_size(n, arity, rows_to_discard) entries, bottom-up; the discarded rows are built in
    // discard_tmp (>= n / arity entries, two ping-pong halves) and dropped
    tree_rows_size(n, arity, rows_to_discard);  // validates the shape
    const fr_t *cur = leaves;
    uint64_t row = n;
    unsigned level = 0;
    fr_t *dst = rows;
    const uint64_t half = n / arity;
    while (row > 1) {
        const uint64_t next = row / arity;
        level++;
        fr_t *o;
        if (level > rows_to_discard) {
            o = dst;
            dst += next;
        } else {
            o = discard_tmp + ((level & 1) ? 0 : half);
        }
        poseidon_hash_dev(c, arity, cur, next, arity, 1, o);
        cur = o;
        row = next;
    }
}

}  // namespace mi
