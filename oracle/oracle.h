/*
 * oracle.h -- CPU restatement of the Groth16/BLS12-381 hot path (TEST INFRASTRUCTURE ONLY).
 *
 * PARITY UNPINNED (task rules): the reference's own prover cannot be built or imported here and its
 * tests hold no golden proof vector.  The oracle is pinned instead by published
 * BLS12-381 constants, an independent pure-Python restatement (tests/golden/pyref.py ->
 * golden.json) and the Groth16 pairing equation.
 *
 * This is the parity oracle for the MI355X proving core.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product library (libfilgpu.so) never links it.
 *
 * What it restates (the reference's hot path lives in un-vendored crypto3 submodules that are
 * empty in /root/reference -- SURVEY.md §0, §8c -- so the algorithm is restated from the
 * public Groth16 / bellman design that the reference's data contracts follow):
 *   - Fq / Fr Montgomery arithmetic          (libs/crypto/multiprecision, [NOT IN TREE])
 *   - BLS12-381 G1 / G2 group law             (libs/crypto/algebra, [NOT IN TREE];
 *                                              curve named at core/crypto/scheme_params.hpp:39-43)
 *   - radix-2 evaluation domain (fft/ifft/coset, generator 7, 2-adicity 32)
 *                                             (libs/crypto/math, [NOT IN TREE])
 *   - Pippenger multiexp                      (libs/crypto/algebra multiexp, [NOT IN TREE])
 *   - Groth16 keygen / prove in the bellman layout of scheme_params{vk,h,l,a,b_g1,b_g2}
 *                                             (core/crypto/scheme_params.hpp:46-66,
 *                                              core/crypto/mapped_scheme_params.hpp:63-81)
 *   - 192-byte proof = compressed A(48) | B(96) | C(48)  (proofs/constants.hpp:93)
 *
 * Wire formats used across this API (all plain bytes):
 *   Fr      : 32 bytes little-endian canonical          (core/fr32.hpp:36-52)
 *   G1 aff  : 96 bytes zcash "uncompressed" big-endian x|y, 0x40 flag in byte 0 = infinity
 *   G2 aff  : 192 bytes x.c1|x.c0|y.c1|y.c0 big-endian, same flags
 *   G1/G2 compressed: 48 / 96 bytes, 0x80 = compressed, 0x40 = infinity, 0x20 = y is largest
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* R1CS in CSR form.  Variables: index 0..num_inputs-1 are inputs (0 is ONE), then aux. */
typedef struct {
    uint64_t num_constraints;
    uint64_t num_inputs;   /* including ONE */
    uint64_t num_aux;
    /* per matrix (A,B,C): row_ptr[num_constraints+1], col[nnz], coeff[nnz*32] (Fr LE canonical) */
    const uint64_t *row_ptr[3];
    const uint32_t *col[3];
    const uint8_t *coeff[3];
} or_r1cs;

/* ---- field / curve known-answer helpers ---- */
void or_fr_mul(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]);
void or_fr_inv(const uint8_t a[32], uint8_t out[32]);
void or_fr_root_of_unity(unsigned log_n, uint8_t out[32]);
void or_g1_generator(uint8_t out96[96]);
void or_g2_generator(uint8_t out192[192]);
int or_g1_mul(const uint8_t p96[96], const uint8_t s[32], uint8_t out96[96]);
int or_g2_mul(const uint8_t p192[192], const uint8_t s[32], uint8_t out192[192]);
int or_g1_add(const uint8_t a96[96], const uint8_t b96[96], uint8_t out96[96]);
int or_g2_add(const uint8_t a192[192], const uint8_t b192[192], uint8_t out192[192]);
int or_g1_compress(const uint8_t p96[96], uint8_t out48[48]);
int or_g2_compress(const uint8_t p192[192], uint8_t out96[96]);
int or_g1_on_curve(const uint8_t p96[96]);
int or_g2_on_curve(const uint8_t p192[192]);

/* fixed-base: out[i] = k[i] * G  (G = standard generator), affine, multi-threaded */
void or_g1_fixed_base(const uint8_t *k32, size_t n, uint8_t *out96);
void or_g2_fixed_base(const uint8_t *k32, size_t n, uint8_t *out192);

/* ---- evaluation domain (bellman EvaluationDomain semantics, natural order in/out) ---- */
/* kind: 0 = fft, 1 = ifft, 2 = coset_fft, 3 = icoset_fft.  n = 2^log_n elements in place. */
void or_ntt(uint8_t *data32, unsigned log_n, int kind);

/* ---- multiexp ---- */
int or_msm_g1(const uint8_t *bases96, const uint8_t *scalars32, size_t n, uint8_t out96[96]);
int or_msm_g2(const uint8_t *bases192, const uint8_t *scalars32, size_t n, uint8_t out192[192]);
int or_msm_g1_naive(const uint8_t *bases96, const uint8_t *scalars32, size_t n, uint8_t out96[96]);

/* ---- Groth16 ---- */
/* Toxic waste: tau, alpha, beta, gamma, delta (Fr LE canonical, 5*32 bytes). */
typedef struct or_params or_params;   /* opaque: vk + h,l,a,b_g1,b_g2 + densities + trapdoor evals */
or_params *or_groth16_keygen(const or_r1cs *cs, const uint8_t toxic[5 * 32]);
void or_params_free(or_params *p);
/* Load externally produced params (wire encodings; densities derived from the R1CS). NULL on error. */
or_params *or_params_from_queries(const or_r1cs *cs, const uint8_t *h, uint64_t n_h, const uint8_t *l,
                                  const uint8_t *a, uint64_t n_a, const uint8_t *b_g1, const uint8_t *b_g2,
                                  uint64_t n_b, const uint8_t *vk, const uint8_t *ic);
/* Sizes of the queries (number of points) */
void or_params_sizes(const or_params *p, uint64_t out[6]); /* d, |h|, |l|, |a|, |b_g1|, |b_g2| */
/* Export the bellman-layout queries: h,l,a,b_g1 as G1 96B, b_g2 as G2 192B, vk (see .cpp) */
void or_params_export(const or_params *p, uint8_t *h, uint8_t *l, uint8_t *a, uint8_t *b_g1,
                      uint8_t *b_g2, uint8_t *vk /* 96*3 + 192*3 = 864 bytes: alpha1,beta1,beta2,gamma2,delta1,delta2 */,
                      uint8_t *ic /* num_inputs*96 */);

/* Bellman prover with injected r, s.  z = inputs (num_inputs*32, [0] must be ONE) ++ aux.
 * proof_out: 192 bytes compressed; raw_out (optional): A 96 | B 192 | C 96 uncompressed;
 * h_out (optional): the (d-1) H coefficients (Fr LE canonical). */
int or_groth16_prove(const or_params *p, const or_r1cs *cs, const uint8_t *z32, const uint8_t r[32],
                     const uint8_t s[32], uint8_t proof_out[192], uint8_t *raw_out, uint8_t *h_out);
/* Trapdoor check: recompute A,B,C from the toxic waste + QAP identity, compare with raw proof.
 * returns 1 when the proof is the unique valid proof for (z, r, s). */
int or_groth16_trapdoor_check(const or_params *p, const or_r1cs *cs, const uint8_t *z32,
                              const uint8_t r[32], const uint8_t s[32], const uint8_t raw[384]);
/* R1CS satisfaction check (1 = satisfied) */
int or_r1cs_satisfied(const or_r1cs *cs, const uint8_t *z32);

/* ---- pairing-based verifier (e(A,B) = e(alpha,beta) e(IC,gamma) e(C,delta)) ---- */
int or_groth16_verify(const uint8_t vk864[864], const uint8_t *ic96, uint64_t num_inputs,
                      const uint8_t *inputs32 /* num_inputs*32 incl. ONE */, const uint8_t raw[384]);

/* threads used by the oracle (OpenMP); 0 = library default */
/* Poseidon, literal form (constants from oracle/poseidon_ref.py); out[i] = hash of in[i*arity ..] */
int or_poseidon_hash(unsigned arity, const uint8_t *rc32, const uint8_t *mds32, unsigned rf, unsigned rp,
                     const uint8_t *in32, uint64_t n, uint8_t *out32);
/* the same in the sparse form (constants from poseidon_ref.sparse_form) */
int or_poseidon_hash_sparse(unsigned arity, unsigned rf, unsigned rp, const uint8_t *first32, const uint8_t *part32,
                            const uint8_t *last32, const uint8_t *mds32, const uint8_t *rows32, const uint8_t *dense32,
                            const uint8_t *in32, uint64_t n, uint8_t *out32);
void or_set_threads(int n);
int or_get_threads(void);

/* SHA-256 (FIPS 180-4) and the SDR labelling witness: labels[i] = SHA256(replica_id || u32_be(layers[i]) ||
 * u64_be(nodes[i]) || 0^20 || 37 parents repeated cyclically from parents[i * n_parents ..]), byte 31 &= 0x3f;
 * n_parents = 0: the prefix alone (node 0) */
void or_sha256(const uint8_t *msg, uint64_t len, uint8_t out[32]);
int or_sdr_labels(const uint8_t replica_id[32], uint64_t count, const uint32_t *layers, const uint64_t *nodes,
                  const uint8_t *parents, unsigned n_parents, uint8_t *labels);

#ifdef __cplusplus
}
#endif
