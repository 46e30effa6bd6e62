// Stacked-PoRep circuit: the R1CS shape of one partition, built on the host once per
// shape, and the witness program the GPU runs per partition.
//
// Reference: StackedCircuit::synthesize (libs/storage/include/nil/filecoin/storage/proofs/porep/stacked/
// circuit/proof.hpp:98-165) and Proof::synthesize (circuit/params.hpp:93-238): the replica id, comm_d and
// comm_r inputs, comm_r = H(comm_c || comm_r_last), then per challenge the tree D inclusion of the data leaf
// (SHA-256), the 6 DRG + 8 expander parent columns hashed (Poseidon) and included in tree C, the challenge
// as a UInt64 input, one create_label SHA-256 gadget per layer over the 37 expanded parents, the encoding
// key + data, and the tree R-last / tree C inclusions of the encoded node and of the column hash.
//
// The gadgets follow bellman / rust-fil-proofs / neptune as oracle/stacked_circuit.py restates them; the
// reference pins the constraint counts (598 per Poseidon-11 column hash, the PoR counts, and 1,199,620 /
// 1,206,212 / 1,296,576 / 1,346,982 for the 2-layer 1-challenge circuit of base 8 / 2 / 8-4 / 8-4-2), and
// tests/test_cpu_stacked_circuit.py checks this builder's R1CS equals the oracle's row for row.
//
// Witness program.  Every variable the synthesis allocates is produced by one op of a small tape:
//   light ops (data copies, bit decompositions, picks, and/nor bits, adds) write all their variables;
//   heavy ops (a Poseidon hash, a SHA-256 hash over many blocks) write their output variable in phase A
//   (a native evaluation) and their internal variables in phase B (the gadget's allocations re-derived
//   from the native round states, one thread per Poseidon hash / per SHA-256 block).
// Phase A runs level by level (level = 1 + the deepest producer of an operand): about 3 levels per tree D
// level and 2 per tree C level.  Phase B is one launch per heavy op kind.
#pragma once
#include <cstdint>
#include <mutex>
#include <utility>
#include <vector>

#include "field.h"

namespace mi {
struct Ctx;
namespace stacked {

struct Shape {
    unsigned layers = 2;       // SDR layers (columns of `layers` labels; 11 at 32 GiB)
    unsigned challenges = 1;   // challenges per partition (18 at 32 GiB: proofs/parameters.hpp:90-99); PoSt:
                               // challenges per sector (Window PoSt: 10)
    uint64_t nodes = 8;        // sector nodes (2^30 at 32 GiB)
    unsigned base = 8, sub = 0, top = 0;  // tree C / tree R-last arities (32 GiB: 8, 8, 0)
    unsigned sectors = 0;      // 0: the stacked PoRep circuit; > 0: the Fallback PoSt circuit over this many
                               // sectors (Window PoSt at 32 GiB: 2349, constants.hpp:85-89)
};

// instance data: an array of 32-byte slots (Fr little-endian canonical; u64 values in the low 8 bytes)
//   global  0 replica_id  1 comm_d  2 comm_r  3 comm_r_last  4 comm_c
//   per challenge c, from 5 + c * stride:
//     +0 challenge index (u64)   +1 data leaf   +2 .. tree D siblings (depth_d, leaf upward)
//     tree R-last siblings (sum over levels of arity - 1, position order, leaf upward)
//     tree C siblings of the challenged column (same count)
//     6 DRG parents, then 8 expander parents, each: index (u64), column (layers labels, layer 1 first),
//     tree C siblings
//
// Fallback PoSt instance (sectors > 0): per sector s, from s * stride:
//   +0 comm_r  +1 comm_c  +2 comm_r_last, then per challenge n, from 3 + n * (2 + path_c):
//     +0 challenged leaf index (u64)  +1 leaf  +2 .. tree R-last siblings (position order, leaf upward)
struct Layout {
    unsigned depth_d = 0;               // binary tree D levels
    std::vector<unsigned> c_arities;    // tree C / R-last level arities, leaf upward
    uint64_t path_c = 0;                // siblings per tree C / R-last path
    uint64_t stride = 0;                // slots per challenge
    uint64_t slots = 0;                 // total slots
    uint64_t unit0 = 5;                 // first slot of the replicated unit (challenge; PoSt: sector 0)
    uint64_t ch_base(unsigned c) const { return 5 + (uint64_t)c * stride; }
    uint64_t post_sector(uint64_t s) const { return s * stride; }
    uint64_t post_challenge(uint64_t s, unsigned n) const { return s * stride + 3 + (uint64_t)n * (2 + path_c); }
    uint64_t off_d() const { return 2; }
    uint64_t off_r() const { return 2 + depth_d; }
    uint64_t off_cx() const { return 2 + depth_d + path_c; }
    uint64_t off_parent(unsigned p, unsigned layers) const {
        return 2 + depth_d + 2 * path_c + (uint64_t)p * (1 + layers + path_c);
    }
};
Layout layout_for(const Shape &s);

enum WopType : uint32_t {
    W_DATA = 0,   // z[dst] = slot a
    W_COPY,       // z[dst] = z[a]
    W_BITS,       // z[dst + i] = bit i of z[a], i < n
    W_DBITS,      // z[dst + i] = bit (b + i) of the u64 in slot a, i < n
    W_DPACK,      // z[dst] = the u64 in slot a, low n bits
    W_PICK,       // z[dst] = z[c] ? z[a] : z[b]
    W_AND,        // z[dst] = z[a] & z[b] (bits)
    W_NOR,        // z[dst] = !z[a] & !z[b]
    W_ADD,        // z[dst] = z[a] + z[b] (mod r)
    W_POSEIDON,   // arity n, inputs z[pin[a .. a + n)], internal variables from dst, digest z[b]
    W_SHA,        // n blocks from blocks[a], internal variables per block, packed 254-bit digest z[b]
};
struct WOp {
    uint32_t type, n, level, pad;
    uint64_t dst, a, b, c;
};
// SHA-256 message words: kind in the top 2 bits
//   0 constant (low 32 bits), 1 bytes 4k..4k+3 of z[v] (v = payload >> 3, k = payload & 7): one word of
//   reverse_bit_numbering(to_bits_le(v)) whose bit 7 is the constant pad bit when k = 7,
//   2 the high (k = 0) / low (k = 1) half of the u64 in slot (payload >> 1) as UInt64::to_bits_be
static constexpr uint64_t WD_CONST = 0, WD_FR = 1ull << 62, WD_U64 = 2ull << 62;
struct ShaBlock {
    uint64_t base;      // first variable of this compression's gadget
    uint64_t desc[16];  // message words
    uint32_t iv;        // 1: the input state is the IV (constant); 0: the previous block's output (allocated)
    uint32_t op;        // index of the W_SHA op
};

struct Built {
    Shape shape;
    Layout lay;
    uint64_t n_in = 0, n_aux = 0, n_constraints = 0;
    // R1CS over z = ONE ++ inputs ++ aux; entry e of matrix m has coefficient ctab[cidx[m][e]] (canonical
    // little-endian fr_t raw limbs; ctab[0] = 1).  A circuit has few distinct coefficients (about 1.5 K for
    // the stacked circuit: powers of two, the Poseidon constants), so an entry costs 8 bytes, not 36.
    std::vector<uint64_t> rp[3];
    std::vector<uint32_t> col[3];
    std::vector<uint32_t> cidx[3];
    std::vector<fr_t> ctab;
    // witness program
    std::vector<WOp> ops;            // sorted by (level, kind): kind 0 every non-Poseidon op, 1..4 Poseidon of
                                     // arity 2 / 4 / 8 / 11 (one kernel per kind)
    std::vector<uint64_t> level_off; // ops of level L: [level_off[L], level_off[L + 1])
    std::vector<uint64_t> seg_off;   // ops of (level L, kind k): [seg_off[5 L + k], seg_off[5 L + k + 1])
    std::vector<uint64_t> pin;       // Poseidon input variable lists
    std::vector<ShaBlock> blocks;
    std::vector<uint64_t> poseidon_ops, sha_ops;  // op indices (phase B)
    // device copies of the program (stacked_witness.hip), one per context (Ctx::uid) that ran the witness,
    // uploaded on first use.  Each holds that context's Poseidon table views and its own SHA chaining-value
    // scratch, so contexts on one or several devices never share device state; calls through one context are
    // serialised by its lock, and dev_mu guards the list itself.
    std::mutex dev_mu;
    std::vector<std::pair<uint64_t, void *>> dev_progs;
    Built() = default;
    Built(const Built &) = delete;
    Built &operator=(const Built &) = delete;
    ~Built();
};

// Builds the R1CS and the witness program of one partition of `s` (throws std::invalid_argument on a shape
// the circuit cannot take: layers 2 or 11 (Poseidon column arity), power-of-two node count matching the
// tree shape, arities in {2, 4, 8}).  With s.sectors > 0 the circuit is FallbackPoStCircuit::synthesize
// (rust-fil-proofs storage-proofs-post fallback/circuit.rs; the reference keeps its data types,
// post/fallback/circuit.hpp:38-86): per sector comm_c, comm_r_last, comm_r (an input), Poseidon-2(comm_c,
// comm_r_last) == comm_r, and one private tree R-last PoR per challenge (path packed into one input).
Built *build(const Shape &s, bool want_r1cs = true);

// generate_public_inputs order (circuit/proof.hpp:186-269; PoSt: per sector comm_r, then the challenged leaf
// index of each inclusion proof) from the instance slots, without ONE
void public_inputs(const Built &b, const uint8_t *slots, std::vector<fr_t> &out);

// The witness of one partition on the GPU: slots_dev = the instance (Layout), z_dev = (n_in + n_aux) x 32 B,
// written completely (z[0] = ONE, the public inputs, every aux variable), canonical little-endian.
// Returns after the last kernel finished (on the context stream).  Phase timings go to c.stats.
void witness_dev(Ctx &c, Built &b, const uint8_t *slots_dev, fr_t *z_dev);
// drops the device programs a context (Ctx::uid) uploaded into every circuit (mi_ctx_destroy)
void forget_ctx(uint64_t uid);

// Poseidon circuit constraint count for one hash (3 per first-round S-box of an input, 4 per later S-box,
// 1 for the digest): 311 / 377 / 505 / 598 for arity 2 / 4 / 8 / 11
uint64_t poseidon_constraints(unsigned arity);

}  // namespace stacked
}  // namespace mi
