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
    MI_UNROLL for (int l = 0; l < 9; l++) s[0].v[l] = k.img[k.off_tag].v[l];
    const fr_t *p = in + i * stride_hash;
    sfor<T - 1>([&](auto j) { s[j + 1] = fr29_mul(fr29_from_fr(p[(uint64_t)j * stride_elem]), r2); });
    out[i] = fr_from_fr29(fr29_from_mont(poseidon_permute<T>(s, k)));
}

// Wave-pair form (default): a 128-thread workgroup hashes 64 inputs; wave 0 holds state elements
// [0, H0) and wave 1 elements [H0, t) of the same 64 hashes (H0 = ceil(t / 2)), and the halves are
// exchanged through LDS around every matrix step.  Each wave's role is uniform, so round constants and
// matrix rows stay scalar loads, and a lane holds half a state plus the partner half and the new half
// (3 x ceil(t/2) x 9 registers: 162 at t = 12) -- two waves per SIMD instead of one for k_poseidon<12>
// (353 registers), which is what hides the dependent product-scanning chains.  Partial rounds exchange
// one element each way: the S-boxed s0 (wave 0 -> 1) and wave 1's half of the sparse row (1 -> 0).
// Every barrier sits in code both waves execute.
template <int T>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) k_poseidon_pair(const fr_t *__restrict__ in, uint64_t n, uint64_t stride_hash,
                                                       uint64_t stride_elem, PosK k, fr_t *__restrict__ out) {
    constexpr int H0 = (T + 1) / 2, H1 = T / 2;
    __shared__ uint32_t xb[2][H0][9][64];
    const unsigned lane = threadIdx.x & 63, role = threadIdx.x >> 6;
    const uint64_t i = (uint64_t)blockIdx.x * 64 + lane;
    const bool live = i < n;
    const fr29_t *img = k.img;
    const fr29_t zero = {{0, 0, 0, 0, 0, 0, 0, 0, 0}};
    fr29_t s[H0], p[H0];
    {
        const fr29_t r2 = img[k.off_tag + 1];
        const fr_t *src = in + (live ? i : 0) * stride_hash;
        if (role == 0) {
            MI_UNROLL for (int l = 0; l < 9; l++) s[0].v[l] = img[k.off_tag].v[l];  // limb-wise: a struct memcpy into s kept it in scratch
            sfor<H0 - 1>([&](auto j) {
                s[j + 1] = live ? fr29_mul(fr29_from_fr(src[(uint64_t)j * stride_elem]), r2) : zero;
            });
        } else {
            sfor<H0>([&](auto j) { s[j] = zero; });
            sfor<H1>([&](auto j) {
                s[j] = live ? fr29_mul(fr29_from_fr(src[(uint64_t)(H0 - 1 + j) * stride_elem]), r2) : zero;
            });
        }
    }
    const int own = role ? H1 : H0, partner = role ? H0 : H1;
    auto put = [&](int cnt) __attribute__((always_inline)) {
        __syncthreads();  // the partner has read the previous exchange
        sfor<H0>([&](auto j) {
            if (j < cnt) MI_UNROLL for (int l = 0; l < 9; l++) xb[role][j][l][lane] = s[j].v[l];
        });
        __syncthreads();
    };
    auto get = [&](int cnt) __attribute__((always_inline)) {
        sfor<H0>([&](auto j) {
            if (j < cnt) MI_UNROLL for (int l = 0; l < 9; l++) p[j].v[l] = xb[role ^ 1][j][l][lane];
        });
    };
    // s <- M s for a t x t matrix (full rounds, dense last partial round)
    auto mat = [&](const fr29_t *__restrict__ m) __attribute__((always_inline)) {
        put(own);
        get(partner);
        if (role == 0) {
            fr29_t nn[H0];
            sfor<H0>([&](auto r) {
                __builtin_amdgcn_sched_barrier(0);  // one row at a time (register pressure)
                nn[r] = fr29_add(fr29_row<H0>(m + r * T, s), fr29_row<H1>(m + r * T + H0, p));
            });
            __builtin_amdgcn_sched_barrier(0);
            sfor<H0>([&](auto r) { s[r] = nn[r]; });
        } else {
            fr29_t nn[H1];
            sfor<H1>([&](auto r) {
                __builtin_amdgcn_sched_barrier(0);
                nn[r] = fr29_add(fr29_row<H1>(m + (H0 + r) * T + H0, s), fr29_row<H0>(m + (H0 + r) * T, p));
            });
            __builtin_amdgcn_sched_barrier(0);
            sfor<H1>([&](auto r) { s[r] = nn[r]; });
        }
    };
    auto full = [&](const fr29_t *__restrict__ rc) __attribute__((always_inline)) {
        if (role == 0)
            sfor<H0>([&](auto j) {
                __builtin_amdgcn_sched_barrier(0);
                s[j] = fr29_sbox(fr29_add(s[j], rc[j]));
            });
        else
            sfor<H1>([&](auto j) {
                __builtin_amdgcn_sched_barrier(0);
                s[j] = fr29_sbox(fr29_add(s[j], rc[H0 + j]));
            });
        __builtin_amdgcn_sched_barrier(0);
        mat(img + k.off_mds);
    };
#pragma unroll 1
    for (int r = 0; r < k.rf / 2; r++) full(img + k.off_rc_first + r * T);
    const fr29_t *sp = img + k.off_sparse;
#pragma unroll 1
    for (int q = 0; q < k.rp - 1; q++, sp += 2 * T - 1) {
        fr29_t d;
        if (role == 0) {
            s[0] = fr29_sbox(fr29_add(s[0], img[k.off_rc_part + q]));
            d = fr29_row<H0>(sp, s);
        } else {
            d = fr29_row<H1>(sp + H0, s);
        }
        __syncthreads();
        MI_UNROLL for (int l = 0; l < 9; l++) xb[role][0][l][lane] = role ? d.v[l] : s[0].v[l];
        __syncthreads();
        fr29_t recv;
        MI_UNROLL for (int l = 0; l < 9; l++) recv.v[l] = xb[role ^ 1][0][l][lane];
        if (role == 0) {  // recv = wave 1's half of the row
            sfor<H0 - 1>([&](auto j) {
                __builtin_amdgcn_sched_barrier(0);
                s[j + 1] = fr29_sub_if_ge(fr29_add(s[j + 1], fr29_mul(sp[T + j], s[0])), R2X29);
            });
            s[0] = fr29_add(d, recv);
        } else {  // recv = S-boxed s0
            sfor<H1>([&](auto j) {
                __builtin_amdgcn_sched_barrier(0);
                s[j] = fr29_sub_if_ge(fr29_add(s[j], fr29_mul(sp[T + H0 - 1 + j], recv)), R2X29);
            });
        }
    }
    if (role == 0) s[0] = fr29_sbox(fr29_add(s[0], img[k.off_rc_part + k.rp - 1]));
    mat(img + k.off_dense);
#pragma unroll 1
    for (int r = 0; r < k.rf / 2; r++) full(img + k.off_rc_last + r * T);
    if (role == 0 && live) out[i] = fr_from_fr29(fr29_from_mont(s[1]));
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
    // tune::POSEIDON_PAIR (A/B): 1 wave-pair kernel, 0 one thread per hash; unset = the measured choice, pairs for
    // the wide states (arity 8, 11) and one thread per hash for arity 2, 4
    const int64_t pt = tune::get(tune::POSEIDON_PAIR, tune::UNSET);
    const bool pair = pt != tune::UNSET ? pt != 0 : arity >= 8;
    const unsigned gp = (unsigned)((n + 63) / 64);
    switch (arity) {
        case 2:
            if (pair) k_poseidon_pair<3><<<gp, 128, 0, c.stream>>>(in, n, stride_hash, stride_elem, k, out);
            else k_poseidon<3><<<grid256(n), 256, 0, c.stream>>>(in, n, stride_hash, stride_elem, k, out);
            break;
        case 4:
            if (pair) k_poseidon_pair<5><<<gp, 128, 0, c.stream>>>(in, n, stride_hash, stride_elem, k, out);
            else k_poseidon<5><<<grid256(n), 256, 0, c.stream>>>(in, n, stride_hash, stride_elem, k, out);
            break;
        case 8:
            if (pair) k_poseidon_pair<9><<<gp, 128, 0, c.stream>>>(in, n, stride_hash, stride_elem, k, out);
            else k_poseidon<9><<<grid256(n), 256, 0, c.stream>>>(in, n, stride_hash, stride_elem, k, out);
            break;
        case 11:
            if (pair) k_poseidon_pair<12><<<gp, 128, 0, c.stream>>>(in, n, stride_hash, stride_elem, k, out);
            else k_poseidon<12><<<grid256(n), 256, 0, c.stream>>>(in, n, stride_hash, stride_elem, k, out);
            break;
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

// ---- inclusion proofs (MerkleTree_gen_proof / gen_cached_proof, vanilla/proof.hpp:139-140,183-186) ----
namespace {
struct RowOffsets {
    uint64_t off[48];  // entry offset in the stored rows of row j (j > rows_to_discard)
};

// blocks[i * B + k] = base[(c_i / B) * B + k]: the aligned arity^(rtd+1)-leaf block holding challenge i
__global__ void __launch_bounds__(256) k_path_blocks(const fr_t *__restrict__ base, const uint64_t *__restrict__ chal,
                                                     uint64_t count, uint64_t B, fr_t *__restrict__ blocks) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count * B) return;
    const uint64_t i = t / B, k = t % B;
    blocks[t] = base[(chal[i] / B) * B + k];
}

// one thread per (challenge, row): the arity - 1 siblings of the challenge's ancestor in row j, in position
// order skipping its own slot; row 0 also writes the leaf
__global__ void __launch_bounds__(256) k_path_siblings(const fr_t *__restrict__ base, const fr_t *__restrict__ stored,
                                                       const fr_t *__restrict__ rec, const uint64_t *__restrict__ chal,
                                                       uint64_t count, uint32_t A, uint32_t H, uint32_t rtd, uint64_t B,
                                                       RowOffsets ro, fr_t *__restrict__ leaf_out,
                                                       fr_t *__restrict__ sib_out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count * H) return;
    const uint64_t i = t / H;
    const uint32_t j = (uint32_t)(t % H);
    const uint64_t c = chal[i];
    uint64_t pw = 1;
    for (uint32_t r = 0; r < j; r++) pw *= A;
    const fr_t *row;
    uint64_t idx;
    if (j == 0) {
        row = base;
        idx = c;
        leaf_out[i] = base[c];
    } else if (j <= rtd) {
        // recomputed row j of challenge i's block: rows of all blocks are contiguous, block i's part at i * B / A^j
        uint64_t roff = 0, rows = count * B;
        for (uint32_t r = 1; r < j; r++) {
            rows /= A;
            roff += rows;
        }
        row = rec + roff + i * (B / pw);
        idx = (c % B) / pw;
    } else {
        row = stored + ro.off[j];
        idx = c / pw;
    }
    const uint64_t g = idx - idx % A;
    const uint32_t own = (uint32_t)(idx % A);
    fr_t *o = sib_out + t * (A - 1);
    for (uint32_t s = 0, k = 0; s < A; s++)
        if (s != own) o[k++] = row[g + s];
}
inline unsigned grid_of(uint64_t n) { return (unsigned)((n + 255) / 256); }
}  // namespace

unsigned tree_height(uint64_t n, unsigned arity) {
    unsigned h = 0;
    while (n > 1) {
        n /= arity;
        h++;
    }
    return h;
}

void tree_paths_dev(Ctx &c, unsigned arity, const fr_t *base, uint64_t n, unsigned rows_to_discard,
                    const fr_t *stored, const uint64_t *chal, uint64_t count, fr_t *rec_tmp, fr_t *leaf_out,
                    fr_t *sib_out) {
    tree_rows_size(n, arity, rows_to_discard);  // validates the shape
    if (!count) return;
    const unsigned H = tree_height(n, arity);
    if (H >= 48) throw std::invalid_argument("tree: too many rows");
    RowOffsets ro{};
    uint64_t off = 0, row = n;
    for (unsigned j = 1; j <= H; j++) {
        row /= arity;
        if (j > rows_to_discard) {
            ro.off[j] = off;
            off += row;
        }
    }
    uint64_t B = 1;
    for (unsigned r = 0; r <= rows_to_discard; r++) B *= arity;
    if (rows_to_discard) {
        // rebuild the discarded rows of each challenge's aligned block (cached-proof regeneration)
        fr_t *blocks = rec_tmp;
        fr_t *dst = rec_tmp + count * B;
        k_path_blocks<<<grid_of(count * B), 256, 0, c.stream>>>(base, chal, count, B, blocks);
        MI_LAUNCHED(c, "k_path_blocks");
        const fr_t *cur = blocks;
        uint64_t m = count * B;
        for (unsigned r = 1; r <= rows_to_discard; r++) {
            m /= arity;
            poseidon_hash_dev(c, arity, cur, m, arity, 1, dst);
            cur = dst;
            dst += m;
        }
    }
    k_path_siblings<<<grid_of(count * H), 256, 0, c.stream>>>(base, stored, rows_to_discard ? rec_tmp + count * B : nullptr, chal, count, arity,
                                                               H, rows_to_discard, B, ro, leaf_out, sib_out);
    MI_LAUNCHED(c, "k_path_siblings");
}

}  // namespace mi
