// poseidon.h -- Poseidon over BLS12-381 Fr and the Poseidon Merkle-tree builders (poseidon.hip).
#pragma once
#include <vector>

#include "ctx.h"
#include "fr29.h"

namespace mi {

// Device view of one arity's constant image (9 x 29-bit Montgomery limbs per element):
//   [off_tag] domain tag 2^arity - 1, [off_tag + 1] R^2 mod r, [off_rc_first] R_F/2 x t full-round
//   constants, [off_rc_part] R_P folded partial-round constants (element 0), [off_rc_last] R_F/2 x t,
//   [off_mds] t x t MDS, [off_sparse] (R_P - 1) x (t + t - 1) sparse rounds (row, then w^), [off_dense]
//   t x t matrix of the last partial round.
struct PosK {
    const fr29_t *img;
    int rf, rp;
    uint32_t off_tag, off_rc_first, off_rc_part, off_rc_last, off_mds, off_sparse, off_dense;
};

struct PoseidonHost {
    unsigned arity = 0, t = 0;
    int rf = 0, rp = 0;
    std::vector<fr29_t> img;
    size_t off_tag = 0, off_rc_first = 0, off_rc_part = 0, off_rc_last = 0, off_mds = 0, off_sparse = 0,
           off_dense = 0;
    std::vector<fr_t> plain_rc, plain_mds;  // canonical (raw) round constants and MDS, unfolded
};

// host derivation (poseidon_math.h: Grain LFSR constants, Cauchy MDS, folded constants, sparse
// factorisation) and the host evaluation of one hash are header-only in poseidon_math.h
// per-ctx cached tables (uploaded on first use); dev (optional) receives the device view
const PoseidonHost &poseidon_tables(Ctx &c, unsigned arity, PosK *dev);
void poseidon_free(Ctx &c);
// out[i] = Poseidon_arity(x_{i,0..arity-1}), x_{i,j} = in[i * stride_hash + j * stride_elem]; canonical Fr
void poseidon_hash_dev(Ctx &c, unsigned arity, const fr_t *in, uint64_t n, uint64_t stride_hash,
                       uint64_t stride_elem, fr_t *out);
// data[i] = key[i] + data[i] mod r (porep encode: replica node = label + sector data node)
void encode_dev(Ctx &c, const fr_t *key, fr_t *data, uint64_t n);
// entries of the cached tree rows above the base (rows_to_discard lowest ones dropped)
uint64_t tree_rows_size(uint64_t leaves, unsigned arity, unsigned rows_to_discard);
// rows: tree_rows_size entries, bottom-up; discard_tmp: >= 2 * (n / arity) entries
unsigned tree_height(uint64_t n, unsigned arity);
// inclusion paths of count challenges: leaf_out[i] = base[c_i]; sib_out[(i * H + j) * (arity - 1) ..] = the
// siblings in row j (0 = base) in position order skipping the path's own slot, H = tree height.  stored:
// the cached rows (tree_rows_size layout); discarded rows are rebuilt per challenge block in rec_tmp
// (>= count * arity^(rtd+1) * 2 entries when rows_to_discard > 0)
void tree_paths_dev(Ctx &c, unsigned arity, const fr_t *base, uint64_t n, unsigned rows_to_discard,
                    const fr_t *stored, const uint64_t *chal, uint64_t count, fr_t *rec_tmp, fr_t *leaf_out,
                    fr_t *sib_out);
void tree_build_dev(Ctx &c, unsigned arity, const fr_t *leaves, uint64_t n, unsigned rows_to_discard, fr_t *rows,
                    fr_t *discard_tmp);

}  // namespace mi
