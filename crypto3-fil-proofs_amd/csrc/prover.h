// prover.h -- device-resident circuit / SRS objects and the Groth16 prover (bellman layout).
#pragma once
#include <stdint.h>

#include <shared_mutex>

#include <vector>

#include "ctx.h"

namespace mi {

// R1CS resident on the device (crypto3 keeps the constraint system inside the proving key;
// bellperson re-synthesises it -- here it is uploaded once per circuit shape, like the SRS).
struct Circuit {
    uint64_t n = 0, n_in = 0, n_aux = 0, d = 0;
    unsigned log_d = 0;
    uint64_t nnz[3] = {0, 0, 0};
    uint64_t *row_ptr[3] = {nullptr, nullptr, nullptr};
    uint32_t *col[3] = {nullptr, nullptr, nullptr};
    // entry e of matrix m has coefficient ctab[cidx[m][e]] (Montgomery; ctab[0] = 1): 8 bytes per entry
    uint32_t *cidx[3] = {nullptr, nullptr, nullptr};
    fr_t *ctab = nullptr;
    uint64_t n_ctab = 0;
    // witness-map work units (k_eval_blocks): block i of matrix m = rows [blk[m][i], blk[m][i + 1]), at most
    // EVAL_BLOCK entries and rows, or one longer row alone
    uint32_t *blk[3] = {nullptr, nullptr, nullptr};
    uint64_t n_blk[3] = {0, 0, 0};
    // density index lists into z (bellman a_aux_density / b_input_density / b_aux_density)
    uint32_t *idx_a = nullptr, *idx_b = nullptr;
    uint64_t n_a = 0, n_b = 0, n_b_in = 0;
    // a_rank[v] = r when aux variable v is A point n_in + r (idx_a[n_in + r] = n_in + v), ~0 without A density: maps
    // the entries of L's MSM plan onto A's points (msm_derive_plan, groth16_sums "A plan derived from L's")
    uint32_t *a_rank = nullptr;
    // the same map in 8 bytes per 32 variables (a MALL-resident 16 MB at 2^26): word 2g = the A-density bits of
    // variables 32g.., word 2g + 1 = the A points before them; rank(v) = prefix + popcount(bits below v)
    uint32_t *a_bits = nullptr;
    ~Circuit();
};

// Groth16 proving key resident on the device (scheme_params{vk,h,l,a,b_g1,b_g2},
// core/crypto/scheme_params.hpp:46-66).  h is stored bit-reversed (h_perm[pos] = h[bitrev(pos)])
// so the H coefficients can be consumed in the NTT's natural bit-reversed output order.
struct Srs {
    uint64_t d = 0;
    unsigned log_d = 0;
    uint64_t n_h = 0, n_l = 0, n_a = 0, n_b = 0, n_ic = 0;
    g1_affine_t *h_perm = nullptr, *l = nullptr, *a = nullptr, *b_g1 = nullptr;
    // 2^128 multiples of h_perm, l and a: the split-mode MSM tables (msm_g1 bases_hi), built at load
    g1_affine_t *h_hi = nullptr, *l_hi = nullptr, *a_hi = nullptr;
    // fixed-base window tables (WinTable, ctx.h) of h_perm, l, a, b_g1 (G1) and b_g2 (G2) for small keys (domain
    // <= 2^21 by default), built at load when they fit: wt[q][w * n_q + i] = 2^(wt_c w) P_i
    void *wt[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    unsigned wt_c = 0;
    uint64_t wt_points(int q) const {
        const uint64_t n[5] = {n_h, n_l, n_a, n_b, n_b};
        return q >= 0 && q < 5 ? n[q] : 0;
    }
    uint64_t wt_bytes(int q) const {
        if (q < 0 || q > 4 || !wt[q]) return 0;
        return wt_points(q) * ((256 + wt_c - 1) / wt_c) * (q == 4 ? sizeof(g2_affine_t) : sizeof(g1_affine_t));
    }
    WinTable wt_of(int q) const {
        WinTable t;
        if (q < 0 || q > 4 || !wt[q]) return t;
        t.p = wt[q];
        t.stride = wt_points(q);
        t.c = wt_c;
        t.nwin = (256 + wt_c - 1) / wt_c;
        return t;
    }
    // the A query gathered into the aux index space (a_aux[v] = the A point of aux variable v, the affine infinity
    // where v has no A density), built at load for subgroup-checked large keys: L and the aux part of A then share
    // ONE GLV plan over z_aux (groth16_sums "shared L/A plan"); the inputs' part of A is a[0, n_in)
    g1_affine_t *a_aux = nullptr;
    bool has_tables() const { return h_hi || l_hi || a_hi || a_aux || wt[0] || wt[1] || wt[2] || wt[3] || wt[4]; }
    g2_affine_t *b_g2 = nullptr;
    g1_affine_t alpha_g1, beta_g1, delta_g1;
    g2_affine_t beta_g2, gamma_g2, delta_g2;
    std::vector<g1_affine_t> ic;
    // trapdoor evaluations (only when generated from known toxic waste): per-variable u,v,w(tau)
    fr_t *at = nullptr, *bt = nullptr, *ct = nullptr;
    uint64_t n_vars = 0;  // length of at / bt / ct
    fr_t toxic[5];
    bool has_trapdoor = false;
    // every query point is known to lie in the prime-order subgroup (generated from toxic waste, or
    // loaded with checked = 1): the condition for the GLV split in auto mode (msm_g1 `subgroup`)
    bool in_subgroup = false;
    // Every live key is registered with its device: a proof that runs out of memory may release the split
    // tables of any key on its device (groth16_sums).  Provers and MSMs over the key's points hold use_mu
    // shared; releasing another key's tables takes it exclusive, and only when no one is using that key.
    int device = -1;
    mutable std::shared_mutex use_mu;
    // out-of-memory releases that took this key's split tables since they were last built (mi_srs_readmit)
    uint64_t tables_dropped = 0;
    explicit Srs(int dev);
    Srs(const Srs &) = delete;
    Srs &operator=(const Srs &) = delete;
    ~Srs();
};

struct R1csHost {
    uint64_t n, n_in, n_aux;
    const uint64_t *row_ptr[3];
    const uint32_t *col[3];
    const uint8_t *coeff[3];
};

// the same R1CS with its coefficients as indices into a table of distinct canonical values (ctab[0] = 1):
// the form the circuit builders produce (stacked.h Built)
struct R1csCompact {
    uint64_t n, n_in, n_aux;
    const uint64_t *row_ptr[3];
    const uint32_t *col[3];
    const uint32_t *cidx[3];
    const fr_t *ctab;  // canonical raw
    uint64_t n_ctab;
};
Circuit *circuit_load(Ctx &c, const R1csHost &cs);  // interns the coefficients, then circuit_load_compact
Circuit *circuit_load_compact(Ctx &c, const R1csCompact &cs);
// rows j < n with (A z)_j (B z)_j != (C z)_j (z canonical, device); *first_bad = the first such row or ~0
uint64_t circuit_check(Ctx &c, const Circuit &C, const fr_t *z_dev, uint64_t *first_bad);

struct SrsHost {
    const uint8_t *vk;  // 864 bytes
    const uint8_t *ic;
    uint64_t n_ic;
    const uint8_t *h, *l, *a, *b_g1, *b_g2;
    uint64_t n_h, n_l, n_a, n_b_g1, n_b_g2;
};
Srs *srs_load(Ctx &c, const Circuit *circ, const SrsHost &h, bool checked);
// Streaming form of srs_load (chunked broadcast receivers): begin takes vk, ic and the query sizes (the
// query pointers of `h` are ignored), part decodes points [first, first + n) of query `which`
// (0 h natural order, 1 l, 2 a, 3 b_g1, 4 b_g2) from host or device memory, end validates and returns the
// key.  abort releases a stream that will not be ended (end and a throwing begin release it themselves).
struct SrsStream {
    Srs *S = nullptr;
    bool checked = false;
    g1_affine_t *hnat = nullptr;  // h in natural order until end permutes it
    void *dst[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    uint64_t n[5] = {0, 0, 0, 0, 0}, filled[5] = {0, 0, 0, 0, 0};
    int *bad = nullptr;  // 5 queries x {malformed, infinity, outside subgroup}
    // the circuit's A density (idx_a, copied at begin: the circuit may be freed before end) for Srs::a_aux
    uint32_t *a_idx = nullptr;
    uint64_t n_in = 0, n_aux = 0;
};
SrsStream *srs_stream_begin(Ctx &c, const Circuit *circ, const SrsHost &h, bool checked);
void srs_stream_part(Ctx &c, SrsStream &st, int which, uint64_t first, const uint8_t *bytes, uint64_t n, bool on_device);
Srs *srs_stream_end(Ctx &c, SrsStream *st);
void srs_stream_abort(SrsStream *st);
Srs *srs_generate(Ctx &c, const Circuit &circ, const fr_t toxic_canonical[5]);

struct ProofPoints {
    g1_affine_t A, C;
    g2_affine_t B;
};
// The five MSM results of one proof: sum_i h_i H_i, sum_i z_aux,i L_i, sum_i z_i A_i, sum_i z_i B1_i (G1) and
// sum_i z_i B2_i (G2).  With world > 1 each is one rank's share: the sum over the rank's contiguous slice
// of every query (h in its bit-reversed device order; single-proof latency mode); the shares of
// all ranks add up to the full sums.
struct ProofSums {  // every sum starts as the identity: a lane that never runs leaves a valid (if wrong) point
    g1_xyzz_t H = g1_xyzz_t::inf(), L = g1_xyzz_t::inf(), A = g1_xyzz_t::inf(), B1 = g1_xyzz_t::inf();
    g2_xyzz_t B2 = g2_xyzz_t::inf();
    // s A and r B1, computed by the lane that produced A / B1 as soon as it has (SumRanges::premul_*), so the
    // assembly after the last lane only adds
    g1_xyzz_t sA = g1_xyzz_t::inf(), rB1 = g1_xyzz_t::inf();
    bool premul = false;
};
// The verifying-key points the assembly adds (scheme_params vk: alpha_g1, beta_g1, beta_g2, delta_g1, delta_g2).
struct AssemblyKey {
    g1_affine_t alpha_g1, beta_g1, delta_g1;
    g2_affine_t beta_g2, delta_g2;
};
// z_dev: (n_in + n_aux) canonical Fr on the device (z[0] must be ONE).  r, s canonical.
ProofPoints groth16_prove(Ctx &c, const Srs &srs, const Circuit &circ, const fr_t *z_dev, const fr_t &r,
                          const fr_t &s);
// rank's share of the MSMs (rank < world): the contiguous slice [n k / W, n (k + 1) / W) of every query; the
// witness map and NTT chain run in full on every rank whose H slice is not empty
ProofSums groth16_sums(Ctx &c, const Srs &srs, const Circuit &circ, const fr_t *z_dev, unsigned rank = 0,
                       unsigned world = 1);
// The MSM sums over explicit ranges [lo, lo + cnt) of the queries 0 H (d - 1 points, the key's bit-reversed h
// order), 1 L (aux variables), 2 A (a query), 3 B (b query: B_G1 and B_G2 over the same range).  Any set of
// ranges that partitions every query gives shares that add up to the whole proof's sums.  The witness map and
// the NTT chain run only when the H range is not empty, so a latency-mode group can compute H on one rank and
// spread L, A and B over the others (fil_groth16.distributed.latency_ranges).
struct SumRanges {
    uint64_t lo[4] = {0, 0, 0, 0}, cnt[4] = {0, 0, 0, 0};
    // whole proofs only: the blinding scalars, so the lanes also return s A and r B1 (ProofSums::premul)
    const fr_t *premul_r = nullptr, *premul_s = nullptr;
};
// h_in (optional): the d H coefficients of mi_groth16_h_coeffs_dev (canonical, bit-reversed); the share then skips
// the witness map and the NTT chain
ProofSums groth16_sums_ranges(Ctx &c, const Srs &srs, const Circuit &circ, const fr_t *z_dev, const SumRanges &rg,
                               const fr_t *h_in = nullptr);
// the witness map + NTT chain alone: out = d canonical H coefficients in the key's bit-reversed h order
void groth16_h_coeffs(Ctx &c, const Circuit &circ, const fr_t *z_dev, fr_t *out);
SumRanges share_ranges(const Circuit &circ, unsigned rank, unsigned world);
// releases the 2^128 split tables of a key (its G1 MSMs then take the GLV split); returns the bytes freed.  The
// caller holds the key exclusively (use_mu) or owns it outright.
uint64_t srs_drop_split_tables(Srs &S);
// After an out-of-memory error: drain the context's lanes, then release the split tables of every key on its
// device that no one is using (`first` before the others; may be null) and the context's idle scratch, except a
// buffer holding `keep`.  Returns the bytes freed.
uint64_t release_for_retry(Ctx &c, const Srs *first, const void *keep);
// rebuilds a key's split tables after an out-of-memory release took them, when they fit under the key-load rule;
// returns the table bytes rebuilt (0: nothing dropped, or still no room)
uint64_t srs_readmit(Ctx &c, Srs &S);
// A = alpha + A_sum + r delta, B = beta + B2_sum + s delta, C = H + L + s A + r B1 - r s delta (host)
ProofPoints groth16_assemble(const AssemblyKey &k, const ProofSums &sums, const fr_t &r, const fr_t &s);
// The assembly's terms that depend on the blinding and the key only (five of its seven host scalar
// multiplications): groth16_prove computes them on a host thread while the device runs the MSMs.
struct BlindTerms {
    g1_xyzz_t A0;  // alpha + r delta (G1)
    g2_xyzz_t B0;  // beta + s delta (G2)
    g1_xyzz_t C0;  // r s delta + s alpha + r beta (G1)
};
BlindTerms groth16_blind_terms(const AssemblyKey &k, const fr_t &r, const fr_t &s);
ProofPoints groth16_finish(const BlindTerms &t, const ProofSums &sums, const fr_t &r, const fr_t &s);
AssemblyKey assembly_key(const Srs &srs);
// share wire format (MI_SHARE_BYTES = 576): H | L | A | B_G1 (96 B each) | B_G2 (192 B), zcash uncompressed
void sums_encode(const ProofSums &sums, uint8_t out[576]);
// sum `count` encoded shares and assemble the proof against the uncompressed vk (verify.hip); throws on a
// share or vk point that does not decode onto the curve
ProofPoints groth16_assemble_shares(const uint8_t *vk, const uint8_t *shares, uint64_t count, const fr_t &r,
                                    const fr_t &s);
// trapdoor dlogs of the unique proof for (z, r, s) (requires srs.has_trapdoor): A, B, C in Fr (canonical)
void groth16_trapdoor_dlogs(Ctx &c, const Srs &srs, const Circuit &circ, const fr_t *z_dev, const fr_t &r,
                            const fr_t &s, fr_t out[3]);

// encodings (host)
void g1_compress(const g1_affine_t &a, uint8_t out[48]);
void g2_compress(const g2_affine_t &a, uint8_t out[96]);
void g1_encode(const g1_affine_t &a, uint8_t out[96]);
void g2_encode(const g2_affine_t &a, uint8_t out[192]);
bool g1_decode_host(const uint8_t in[96], g1_affine_t &out);
bool g2_decode_host(const uint8_t in[192], g2_affine_t &out);
fr_t fr_from_le(const uint8_t in[32]);  // canonical raw (not Montgomery)

// Groth16 verification on the host (verify.hip).  vk: MI_VK_BYTES uncompressed, ic: n_ic x 96 B,
// inputs: (n_ic - 1) x 32 B LE canonical (without the implicit ONE), proof: 192 B compressed.
// Throws std::domain_error for undecodable / off-curve / non-subgroup points.
bool groth16_verify(const uint8_t *vk, const uint8_t *ic, uint64_t n_ic, const uint8_t *inputs,
                    const uint8_t proof[192]);
bool groth16_verify_batch(const uint8_t *vk, const uint8_t *ic, uint64_t n_ic, uint64_t count, const uint8_t *inputs,
                          const uint8_t *proofs, const uint8_t *seed32);
void pairing_host(const g1_affine_t &p, const g2_affine_t &q, fq_t out[12]);
void fr_to_le(const fr_t &raw, uint8_t out[32]);

}  // namespace mi
