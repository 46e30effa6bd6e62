/*
 * mi355x_groth16.h -- C ABI of the MI355X-native Groth16 proving core (libfilgpu.so).
 *
 * Drop-in boundary for the crypto3 prover call that NilFoundation/crypto3-fil-proofs makes inside
 * its compound-proof partition loop.  Every entry point below names the reference interface it
 * replaces (paths relative to the reference root; the crypto3 prover itself lives in the empty
 * libs/crypto/zk submodule, .gitmodules:19-21, and is marked [NOT IN TREE]):
 *
 *   mi_groth16_prove        <- crypto3::zk::snark::prove<r1cs_gg_ppzksnark<bls12<381>>>(pk, primary, aux)
 *                              as called per partition by compound_proof::circuit_proofs / prove
 *                              (libs/storage/include/nil/filecoin/storage/proofs/core/proof/
 *                               compound_proof.hpp:89-95,127-137); proof bytes are the 192-byte
 *                              SINGLE_PARTITION_PROOF_LEN record (libs/filecoin/include/nil/filecoin/
 *                              proofs/constants.hpp:93) written by seal_commit_phase2
 *                              (libs/filecoin/include/nil/filecoin/proofs/api/seal.hpp:306-308)
 *   mi_srs_load             <- the proving key behind r1cs_gg_ppzksnark_mapped_scheme_params /
 *                              scheme_params{vk,h,l,a,b_g1,b_g2}
 *                              (core/crypto/scheme_params.hpp:38-67, core/crypto/mapped_scheme_params.hpp:43-84)
 *                              memoised by GROTH_PARAM_MEMORY_CACHE (proofs/caches.hpp:48-67)
 *   mi_srs_generate         <- groth16::generate_random_parameters (core/parameter_cache.hpp:185-200),
 *                              "used for testing only, or where parameters are otherwise unavailable"
 *                              (compound_proof.hpp:171-186)
 *   mi_circuit_load         <- the constraint system held by the crypto3 proving key
 *                              (r1cs_gg_ppzksnark_proving_key::constraint_system, [NOT IN TREE]),
 *                              synthesised by e.g. StackedCompound::circuit (porep/stacked/circuit/proof.hpp:271-299)
 *   mi_msm_g1 / mi_msm_g2   <- crypto3 algebra multiexp ([NOT IN TREE], libs/crypto/algebra)
 *   mi_ntt_fr               <- crypto3 math evaluation_domain fft/ifft/coset ([NOT IN TREE], libs/crypto/math)
 *
 * Conventions
 *   Fr scalars      : 32 bytes little-endian canonical (< r)    (core/fr32.hpp:36-52)
 *   G1 / G2 points  : zcash/bellman "uncompressed" big-endian, 96 / 192 bytes,
 *                     G2 as x.c1|x.c0|y.c1|y.c0, flag 0x40 in byte 0 = infinity
 *   proofs          : compressed A (48) | B (96) | C (48) = 192 bytes
 *   variables       : z = inputs (z[0] = ONE) ++ aux, the crypto3 primary/auxiliary split
 *   status codes    : 0 = OK, < 0 = error (see MI_ERR_*); mi_last_error() has the message
 *                     (thread-local).  The C++ wrapper rethrows these as exceptions, matching the
 *                     reference's assert/throw style (compound_proof.hpp:94).
 *   threading       : a context is internally serialised (one mutex); drive one context per GPU
 *                     from one host thread each for multi-GPU.
 *   device pointers : the entries that take or fill caller device memory (every *_dev entry,
 *                     mi_groth16_trapdoor_dlogs, mi_srs_stream_part with on_device != 0) follow one
 *                     stream-ordering rule, so the caller needs no host synchronisation around them:
 *                     (1) on entry, the library's first device access waits ON THE DEVICE for all work
 *                         queued before the call on the context's caller stream (mi_ctx_set_caller_stream;
 *                         default NULL = the legacy default stream, which by HIP semantics also covers
 *                         every blocking stream -- e.g. torch's default stream).  A producer that fills an
 *                         input or clears an output on its own non-blocking stream names that stream;
 *                     (2) on return, every device output is fully written and no input is read any more,
 *                         so the caller may consume or overwrite them from any stream.
 *                     The library's own streams are non-blocking; they never wait for the NULL stream
 *                     implicitly (the round-4 tree-C race: a torch.zeros fill of the output landed after
 *                     the kernel's writes), which is why rule (1) records an event on the caller stream.
 */
#ifndef MI355X_GROTH16_H
#define MI355X_GROTH16_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MI_OK 0
#define MI_ERR_ARG (-1)
#define MI_ERR_HIP (-2)
#define MI_ERR_INVALID_POINT (-3)
#define MI_ERR_SIZE (-4)
#define MI_ERR_INTERNAL (-5)
#define MI_ERR_NO_DEVICE (-6)

#define MI_PROOF_BYTES 192
#define MI_SHARE_BYTES 576 /* mi_groth16_prove_share: H | L | A | B_G1 (96 B each) | B_G2 (192 B) */
#define MI_VK_BYTES 864 /* alpha_g1 | beta_g1 | beta_g2 | gamma_g2 | delta_g1 | delta_g2 (uncompressed) */

typedef struct mi_ctx mi_ctx;         /* one per GPU: stream, twiddle tables, scratch */
typedef struct mi_circuit mi_circuit; /* device-resident R1CS (one per circuit shape) */
typedef struct mi_srs mi_srs;         /* device-resident proving key (one per circuit shape) */
typedef struct mi_points mi_points;   /* device-resident MSM bases */

/* R1CS in CSR form over variables z = inputs ++ aux (num_inputs includes ONE). */
typedef struct {
    uint64_t num_constraints;
    uint64_t num_inputs;
    uint64_t num_aux;
    const uint64_t *row_ptr[3]; /* A, B, C: num_constraints + 1 offsets each */
    const uint32_t *col[3];     /* variable index per entry */
    const uint8_t *coeff[3];    /* Fr coefficient per entry, 32 B LE */
} mi_r1cs;

/* Proving key in the bellman/filecoin params layout (uncompressed points). */
typedef struct {
    const uint8_t *vk; /* MI_VK_BYTES */
    const uint8_t *ic;
    uint64_t n_ic; /* == num_inputs */
    const uint8_t *h;
    uint64_t n_h; /* d - 1 */
    const uint8_t *l;
    uint64_t n_l; /* num_aux */
    const uint8_t *a;
    uint64_t n_a; /* inputs + aux with A-density */
    const uint8_t *b_g1;
    uint64_t n_b_g1; /* inputs/aux with B-density */
    const uint8_t *b_g2; /* 192-byte points */
    uint64_t n_b_g2;
} mi_srs_host;

/* ---- context ---- */
int mi_device_count(int *out);
int mi_ctx_create(int device, mi_ctx **out);
void mi_ctx_destroy(mi_ctx *ctx);
const char *mi_last_error(void);
/* stream handle (hipStream_t) the context launches on; external work may be ordered against it */
int mi_ctx_stream(mi_ctx *ctx, void **stream_out);
/* the caller stream of the "device pointers" rule above (a hipStream_t on this context's device; NULL = legacy
 * default stream); it stays set for every later call on the context.  The setting belongs to the context, not to
 * the calling thread: a context shared by several host threads that use different caller streams must serialise
 * each (set, entry) pair itself -- the "threading" rule above (one host thread per context) avoids the question */
int mi_ctx_set_caller_stream(mi_ctx *ctx, void *stream);
int mi_ctx_synchronize(mi_ctx *ctx);
/* Page-locked host memory for witnesses.  The reference hands the prover host-side assignments
 * (api/seal.hpp:298-301); a synthesiser that writes z into such a buffer lets the prover's H2D copy
 * run at full DMA rate, and mi_groth16_prove_batch overlaps partition k + 1's copy with partition k's
 * proof.  Pageable witnesses work too (staged through pinned buffers). */
int mi_host_alloc(uint64_t bytes, void **out);
void mi_host_free(void *p);

/* ---- circuits and proving keys ---- */
int mi_circuit_load(mi_ctx *ctx, const mi_r1cs *cs, mi_circuit **out);
/* out: num_constraints, num_inputs, num_aux, d, |a|, |b|, nnz(A), nnz(B), nnz(C) */
int mi_circuit_info(const mi_circuit *c, uint64_t out[9]);
void mi_circuit_free(mi_circuit *c);

/* Every point is decoded with zcash/bellman from_uncompressed rules (flag bits, canonical coordinates,
 * on the curve) and, like bellman's Parameters::read, a point at infinity in h, l, a, b_g1, b_g2 or ic
 * is refused.  checked != 0 (Parameters::read(checked = true), mapped_scheme_params::checked)
 * additionally verifies r * P == O for every point (prime-order subgroup).  Failures: MI_ERR_ARG. */
int mi_srs_load(mi_ctx *ctx, const mi_circuit *circuit_or_null, const mi_srs_host *host, int checked,
                mi_srs **out);
/* Streaming key load (a key broadcast over RCCL arrives in chunks; no rank holds it whole in host memory):
 * begin with vk, ic and counts = |h|, |l|, |a|, |b_g1|, |b_g2|; then every query in order as chunks of
 * wire-format points [first, first + n_points) (query `which` 0 h natural order, 1 l, 2 a, 3 b_g1, 4 b_g2),
 * read from host memory or, with on_device != 0, from device memory on this context's GPU (a received
 * broadcast buffer, decoded in place); the chunk may be reused when the call returns.  end applies the
 * same rules as mi_srs_load and consumes the stream (also on failure); abort discards one. */
typedef struct mi_srs_stream mi_srs_stream;
int mi_srs_stream_begin(mi_ctx *ctx, const mi_circuit *circuit_or_null, const uint8_t *vk, const uint8_t *ic,
                        uint64_t n_ic, const uint64_t counts[5], int checked, mi_srs_stream **out);
int mi_srs_stream_part(mi_srs_stream *st, int which, uint64_t first, const void *bytes, uint64_t n_points,
                       int on_device);
int mi_srs_stream_end(mi_srs_stream *st, mi_srs **out);
void mi_srs_stream_abort(mi_srs_stream *st);
/* toxic waste tau, alpha, beta, gamma, delta: 5 x 32 B LE canonical; generators = standard G1/G2 */
int mi_srs_generate(mi_ctx *ctx, const mi_circuit *circuit, const uint8_t toxic[160], mi_srs **out);
/* vk (MI_VK_BYTES) and ic (num_inputs x 96 B) of a loaded / generated key */
int mi_srs_export_vk(const mi_srs *srs, uint8_t *vk_out, uint8_t *ic_out);
/* download one query in the wire format: which = 0 h (natural order), 1 l, 2 a, 3 b_g1, 4 b_g2 */
int mi_srs_export_query(mi_ctx *ctx, const mi_srs *srs, int which, uint8_t *out, uint64_t cap_points);
/* points [first, first + n) of one query in the wire format, written to device memory (the broadcast source) */
int mi_srs_export_query_dev(mi_ctx *ctx, const mi_srs *srs, int which, uint64_t first, uint64_t n, void *dev_out);
/* sizes: d, |h|, |l|, |a|, |b|, |ic| */
int mi_srs_info(const mi_srs *srs, uint64_t out[6]);
/* G1 MSM mode of a key: out[0] = 1 when the 2^128 split tables of h, l, a are resident (built at load
 * unless MI_MSM_GLV=1 or they would take more than half of the free HBM), out[1] = 1 when every point is
 * known to be in the prime-order subgroup (generated key or checked load).  Without tables, the G1
 * MSMs of a subgroup-known key take the GLV split; otherwise they run the plain 256-bit path. */
int mi_srs_msm_info(const mi_srs *srs, uint64_t out[2]);
/* Split tables after memory pressure: a proof, key generation or key load that runs out of HBM releases the 2^128
 * tables of the device's idle keys and retries (mi_ctx_get_fallbacks); the key then proves through the GLV split,
 * byte-identical.  mi_srs_table_state: out[0] = tables resident, out[1] = releases since they were last built,
 * out[2] = subgroup-known.  mi_srs_readmit rebuilds released tables once they fit again under the key-load rule
 * (e.g. after another key was freed); *rebuilt_bytes (may be NULL) = table bytes rebuilt, 0 when nothing was
 * released or there is still no room.  Waits for proofs running on the key. */
int mi_srs_table_state(const mi_srs *srs, uint64_t out[3]);
/* fixed-base window tables of a small key's G1 queries (built at load / generation when the domain is <= 2^21 and
 * they fit; mi_points_precompute explains them): out[0] window bits, out[1] windows, out[2] queries with a table
 * (0..5: h, l, a, b_g1, b_g2).  Out-of-memory releases take them like the split tables, and mi_srs_readmit rebuilds them. */
int mi_srs_window_tables(const mi_srs *srs, uint64_t out[3]);
/* the shared L/A plan of large subgroup keys: *present = 1 when the key holds its A query gathered into the aux index
 * space (built at load / generation when it fits, next to the split tables' admission rule), so a whole proof's L and
 * A MSMs run over one plan (the inputs' part of A as a small MSM of its own); an out-of-memory release drops it like
 * the tables (the retry runs L and A over plans of their own) and mi_srs_readmit does not rebuild it.  The MSM sums,
 * and so the proof bytes, are those of separate plans.  No reference counterpart (bellman runs the L and A multiexps
 * one after the other, over the same z). */
int mi_srs_shared_la(const mi_srs *srs, int *present);
int mi_srs_readmit(mi_ctx *ctx, mi_srs *srs, uint64_t *rebuilt_bytes);
void mi_srs_free(mi_srs *srs);

/* ---- verification (host CPU; no device needed) ----
 *   mi_groth16_verify       <- crypto3 r1cs_gg_ppzksnark verify / bellman verify_proof, used by the
 *                              self-check of every C2 proof (api/seal.hpp:310-313) and verify_seal
 *   mi_groth16_verify_batch <- bellman verify_proofs_batch behind verify_batch_seal (api/seal.hpp:339-485):
 *                              one multi-pairing over random 128-bit weights drawn from getrandom()
 *                              (bellman: OsRng); soundness against adversarial proofs needs weights the
 *                              prover cannot predict
 *   mi_groth16_verify_batch_seeded  the same with the weights from a ChaCha20 stream keyed by seed32:
 *                              reproducible, for tests only (a known seed lets a forger cancel terms)
 * vk: MI_VK_BYTES, ic: n_ic x 96 B (uncompressed); inputs: (n_ic - 1) x 32 B LE canonical public
 * inputs WITHOUT the implicit ONE (generate_public_inputs order), per proof; proofs: 192 B each.
 * *valid = 1 / 0.  Undecodable, off-curve or non-subgroup proof points: MI_ERR_INVALID_POINT;
 * non-canonical inputs: MI_ERR_ARG.
 *   mi_pairing              <- the reduced optimal-ate pairing e(P, Q) (tests: bilinearity); out =
 *                              12 x 48 B big-endian Fq coefficients on the basis w^0..w^5 (Fq2 = c0, c1). */
int mi_groth16_verify(const uint8_t *vk, const uint8_t *ic, uint64_t n_ic, const uint8_t *inputs,
                      const uint8_t proof[MI_PROOF_BYTES], int *valid);
int mi_groth16_verify_batch(const uint8_t *vk, const uint8_t *ic, uint64_t n_ic, uint64_t count,
                            const uint8_t *inputs, const uint8_t *proofs, int *valid);
int mi_groth16_verify_batch_seeded(const uint8_t *vk, const uint8_t *ic, uint64_t n_ic, uint64_t count,
                                   const uint8_t *inputs, const uint8_t *proofs, const uint8_t seed32[32],
                                   int *valid);
int mi_pairing(const uint8_t g1_96[96], const uint8_t g2_192[192], uint8_t out[576]);

/* ---- parameter files (bellman Parameters::write layout = filecoin v28-*.params) ----
 *   mi_params_inspect <- the header walk of mapped_scheme_params::build_mapped_parameters
 *                        (core/crypto/mapped_scheme_params.hpp:43-84); no device needed:
 *                        out = n_ic, n_h, n_l, n_a, n_b_g1, n_b_g2
 *   mi_params_load    <- read_cached_params / get_groth_params (core/parameter_cache.hpp:125-129,185-200):
 *                        mmap + upload once, resident on the device; checked -> point validation
 *   mi_params_write   <- write_cached_params (core/parameter_cache.hpp:146-152; bellman Parameters::write)
 *   mi_vk_write       <- write_cached_verifying_key (core/parameter_cache.hpp:136-144; bellman VerifyingKey::write: vk | u32 BE n_ic | ic)
 * Malformed files (truncated, trailing bytes) fail with MI_ERR_ARG. */
int mi_params_inspect(const char *path, uint64_t out[6]);
int mi_params_load(mi_ctx *ctx, const mi_circuit *circuit_or_null, const char *path, int checked,
                   mi_srs **out);
int mi_params_write(mi_ctx *ctx, const mi_srs *srs, const char *path);
int mi_vk_write(const mi_srs *srs, const char *path);

/* ---- parameter cache (core/parameter_cache.hpp:50-219) ----
 *   mi_param_cache_id       <- cacheable_parameters::cache_identifier (:166-171): "<cache_prefix>-<hex sha256(identifier)>",
 *                              identifier = pub_params.identifier() (e.g. stacked/vanilla/params.hpp:80-85)
 *   mi_param_cache_path     <- parameter_cache_{params,metadata,verifying_key}_path (:78-94): kind 0 / 1 / 2 ->
 *                              $FIL_PROOFS_PARAMETER_CACHE/v28-<id>.params / .meta / .vk (PARAMETER_CACHE_DIR,
 *                              "/var/tmp/filecoin-proof-parameters/", when the variable is unset)
 *   mi_param_cache_metadata <- get_param_metadata (:173-183): reads <id>.meta, else writes {"sector_size":N};
 *                              *sector_size_out = the cached value
 *   mi_get_groth_params     <- get_groth_params (:185-200) + get_verifying_key (:202-219): loads <id>.params when it
 *                              exists and parses, else generates the key (toxic waste as for mi_srs_generate, or drawn
 *                              from getrandom() when toxic_or_null is NULL), writes <id>.params (atomically, via a
 *                              rename) and <id>.vk when missing; *generated = 1 on that branch.  The cache
 *                              directory must exist (ensure_ancestor_dirs_exist, :96-103): MI_ERR_ARG otherwise.
 * These need no device except mi_get_groth_params. */
#define MI_PARAMS_VERSION 28
int mi_param_cache_id(const char *cache_prefix, const char *identifier, char *out, size_t cap);
int mi_param_cache_path(const char *id, int kind, char *out, size_t cap);
int mi_param_cache_metadata(const char *id, uint64_t sector_size, uint64_t *sector_size_out);
int mi_get_groth_params(mi_ctx *ctx, const mi_circuit *circuit, const char *id, const uint8_t *toxic_or_null,
                        int checked, mi_srs **out, int *generated);

/* ---- Groth16 ---- */
/* z: (num_inputs + num_aux) x 32 B, z[0] = ONE.  Every entry must be canonical (< r): a witness holding
 * a non-canonical entry is refused with MI_ERR_ARG (an Fr32 "MUST represent a valid Fr",
 * core/fr32.hpp:36-40), for host and device witnesses alike.  r, s: injected blinding (tests / parity);
 * priority != 0 runs on the context's high-priority stream (post_config.priority,
 * libs/filecoin/include/nil/filecoin/proofs/types/post_config.hpp:41-42).
 * raw_out (optional, may be NULL): uncompressed A (96) | B (192) | C (96). */
int mi_groth16_prove(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circuit, const uint8_t *z,
                     const uint8_t r[32], const uint8_t s[32], int priority, uint8_t proof_out[MI_PROOF_BYTES],
                     uint8_t *raw_out);
/* same with z already resident in device memory (32 B LE canonical per variable) */
int mi_groth16_prove_dev(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circuit, const void *z_dev,
                         const uint8_t r[32], const uint8_t s[32], int priority, uint8_t proof_out[MI_PROOF_BYTES],
                         uint8_t *raw_out);
/* count independent partitions (compound_proof::circuit_proofs loop); proofs_out = count x 192 B.
 * Partition k + 1's witness upload overlaps partition k's proof (copy stream, two device slots). */
int mi_groth16_prove_batch(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circuit, uint64_t count,
                           const uint8_t *const *z, const uint8_t *rs /* count x 64 B: r | s */, int priority,
                           uint8_t *proofs_out);
/* Production entries with internal randomness (crypto3 prove / bellman create_random_proof: r, s drawn by
 * the prover, never supplied by the caller): r, s uniform in [0, r) from getrandom(), wiped after use.
 * These are what compound_proof::circuit_proofs binds; the injected-(r, s) entries
 * above are the parity/test entries (they accept r = s = 0, which drops zero-knowledge). */
int mi_groth16_prove_random(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circuit, const uint8_t *z,
                            int priority, uint8_t proof_out[MI_PROOF_BYTES]);
int mi_groth16_prove_dev_random(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circuit, const void *z_dev,
                                int priority, uint8_t proof_out[MI_PROOF_BYTES]);
int mi_groth16_prove_batch_random(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circuit, uint64_t count,
                                  const uint8_t *const *z, int priority, uint8_t *proofs_out);
/* Single-proof latency mode (one proof split over `world` GPUs).  Rank `rank` runs the
 * witness map and NTT chain in full and the MSMs over its contiguous slice of each query (h in the
 * bit-reversed coefficient order the device keeps it in; l, a, b_g1/b_g2 in key order), writing the five partial sums, zcash-uncompressed, to share_out.  The callers exchange
 * the shares (an all-gather of MI_SHARE_BYTES per rank) and any of them calls mi_groth16_assemble,
 * which adds the shares and applies the blinding exactly as mi_groth16_prove does: the proof bytes are
 * identical for every world size.  Replaces the single crypto3 prove call of compound_proof::prove
 * (compound_proof.hpp:89-95) when one partition must finish sooner than one GPU can prove it. */
int mi_groth16_prove_share(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circuit, const uint8_t *z,
                           uint32_t rank, uint32_t world, int priority, uint8_t share_out[MI_SHARE_BYTES]);
int mi_groth16_prove_share_dev(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circuit, const void *z_dev,
                               uint32_t rank, uint32_t world, int priority, uint8_t share_out[MI_SHARE_BYTES]);
/* A share over explicit query ranges: ranges[2q], ranges[2q + 1] = first point, count of query q = 0 H (the
 * d - 1 points in the key's bit-reversed h order), 1 L (aux), 2 A (a query), 3 B (b query; B_G1 and B_G2 over
 * the same range).  The witness map and the NTT chain run only when the H count is non-zero, so a latency-mode
 * group computes H once (on the rank that holds the whole H range) and spreads L, A and B over the others;
 * shares whose ranges partition every query assemble into the proof mi_groth16_prove makes. */
int mi_groth16_prove_share_ranges(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circuit, const uint8_t *z,
                                  const uint64_t ranges[8], int priority, uint8_t share_out[MI_SHARE_BYTES]);
int mi_groth16_prove_share_ranges_dev(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circuit, const void *z_dev,
                                      const uint64_t ranges[8], int priority, uint8_t share_out[MI_SHARE_BYTES]);
/* H computed once and SPLIT over a latency group: mi_groth16_h_coeffs_dev runs the witness map and the QAP's NTT chain
 * alone and writes the d canonical H coefficients (32 B LE each, in the key's bit-reversed h order) to h_out_dev;
 * the group broadcasts them (RCCL), and every rank's mi_groth16_prove_share_ranges_h_dev then runs its H slice from
 * h_dev (NULL: computed in place, as mi_groth16_prove_share_ranges_dev) beside its L, A, B slices.  A rank may make
 * several shares (e.g. L/A/B while H is still on its way, then its H slice); mi_groth16_assemble adds them all. */
int mi_groth16_h_coeffs_dev(mi_ctx *ctx, const mi_circuit *circuit, const void *z_dev, void *h_out_dev);
int mi_groth16_prove_share_ranges_h_dev(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circuit, const void *z_dev,
                                        const void *h_dev, const uint64_t ranges[8], int priority,
                                        uint8_t share_out[MI_SHARE_BYTES]);
/* host only (no device): vk = MI_VK_BYTES uncompressed, shares = count x MI_SHARE_BYTES (any order) */
int mi_groth16_assemble(const uint8_t *vk, const uint8_t *shares, uint64_t count, const uint8_t r[32],
                        const uint8_t s[32], uint8_t proof_out[MI_PROOF_BYTES], uint8_t *raw_out);
/* discrete logs (canonical Fr, 3 x 32 B) of the unique valid A, B, C for (z, r, s) under a key
 * produced by mi_srs_generate -- the size-independent trapdoor check used by the tests */
int mi_groth16_trapdoor_dlogs(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circuit, const void *z_dev,
                              const uint8_t r[32], const uint8_t s[32], uint8_t out[96]);

/* ---- building blocks ---- */
int mi_msm_g1(mi_ctx *ctx, const uint8_t *bases96, const uint8_t *scalars32, uint64_t n, uint8_t out96[96]);
int mi_msm_g2(mi_ctx *ctx, const uint8_t *bases192, const uint8_t *scalars32, uint64_t n, uint8_t out192[192]);
/* bellman EvaluationDomain semantics, natural order in and out: (inverse, coset) =
 * (0,0) fft, (1,0) ifft, (0,1) coset_fft, (1,1) icoset_fft.  data: 2^log_n x 32 B, in place. */
int mi_ntt_fr(mi_ctx *ctx, uint8_t *data32, unsigned log_n, int inverse, int coset);

/* device-resident variants: bases uploaded once, scalars / data already in device memory */
int mi_points_upload_g1(mi_ctx *ctx, const uint8_t *bases96, uint64_t n, mi_points **out);
int mi_points_upload_g2(mi_ctx *ctx, const uint8_t *bases192, uint64_t n, mi_points **out);
/* device copies of a generated key's queries (for MSM benchmarking on real SRS points) */
int mi_points_from_srs(mi_ctx *ctx, const mi_srs *srs, int which, mi_points **out);
void mi_points_free(mi_points *p);
/* r P == O for every point (the checked-load test); on success the bases are marked subgroup-known so that
 * large G1 MSMs over them may take the GLV split (phi(P) = lambda P holds only on the r-torsion).  A point
 * outside the subgroup: MI_ERR_ARG, and the bases stay on the exact plain path. */
int mi_points_check_subgroup(mi_ctx *ctx, mi_points *p);
/* out: count, has a 2^128 split table, subgroup-known */
int mi_points_info(const mi_points *p, uint64_t out[3]);
uint64_t mi_points_count(const mi_points *p);
/* Fixed-base window table of the first n_points G1 or G2 bases: T[w n + i] = 2^(c w) P_i, w < ceil(256 / c)
 * (window_bits = c, 0 = the library's choice for n_points).  Later mi_msm_g1_dev / _g2_dev calls over <= n_points
 * scalars run every window's digits into one set of 2^(c - 1) buckets (fewer reductions, no window combination,
 * same result).  Costs ceil(256 / c) x the bases' memory; replaces a previous table.  A proving key's small
 * queries carry tables of their own (built at key load, domain <= 2^21); a table built on a key query's point set
 * (mi_points_from_srs) belongs to that point set and takes precedence for its MSMs.  No reference counterpart: the
 * reference's multiexp (bellman / crypto3 algebra, [NOT IN TREE]) re-reads the same SRS bases on every proof. */
int mi_points_precompute(mi_ctx *ctx, mi_points *p, unsigned window_bits, uint64_t n_points);
/* out: window bits, windows, table points (all 0 without a table) */
int mi_points_table_info(const mi_points *p, uint64_t out[3]);
int mi_msm_g1_dev(mi_ctx *ctx, const mi_points *bases, const void *scalars_dev, uint64_t n, uint8_t out96[96]);
int mi_msm_g2_dev(mi_ctx *ctx, const mi_points *bases, const void *scalars_dev, uint64_t n, uint8_t out192[192]);
int mi_ntt_fr_dev(mi_ctx *ctx, void *data_dev, unsigned log_n, int inverse, int coset);

/* ---- synthetic workload (BASELINE configs 3/4: "synthetic 2^k-constraint R1CS") ----
 * Host-side, deterministic, multithreaded generator of a satisfiable R1CS with 2^log_rows - num_inputs
 * rows (so the evaluation domain is exactly 2^log_rows) and its witness.  Stands in for circuit
 * synthesis (StackedCircuit::synthesize, porep/stacked/circuit/proof.hpp:98-165), which is outside
 * the prover boundary.  Pointers returned by mi_synth_r1cs / mi_synth_witness live until mi_synth_free. */
typedef struct mi_synth mi_synth;
int mi_synth_generate(unsigned log_rows, uint64_t num_inputs, uint64_t seed, mi_synth **out);
/* flags: MI_SYNTH_UNIFORM_WITNESS turns the generator's boolean rows into packing rows, so every aux value is
 * a uniform field element or a product of such (no small MSM scalars: the uniform-witness prove rate) */
#define MI_SYNTH_UNIFORM_WITNESS 1u
int mi_synth_generate_ex(unsigned log_rows, uint64_t num_inputs, uint64_t seed, unsigned flags, mi_synth **out);
int mi_synth_r1cs(const mi_synth *s, mi_r1cs *out);
int mi_synth_witness(const mi_synth *s, const uint8_t **z, uint64_t *num_vars);
void mi_synth_free(mi_synth *s);

/* ---- stacked-PoRep circuit: R1CS and GPU witness generation -----------------------
 * Replaces the synthesis half of compound_proof::circuit_proofs (StackedCompound::circuit + synthesize:
 * libs/storage/include/nil/filecoin/storage/proofs/porep/stacked/circuit/proof.hpp:98-165, params.hpp:93-238):
 *   mi_stacked_build   <- the circuit shape (blank-circuit synthesis): the R1CS of one partition over
 *                         z = ONE ++ inputs ++ aux, identical for every partition of a shape, and the witness
 *                         program.  layers 2 or 11, nodes a power of two, tree C / R-last arities in {2, 4, 8}
 *                         (32 GiB: layers 11, challenges 18, nodes 2^30, 8 / 8 / 0).  Host, no device needed.
 *   mi_stacked_witness <- the assignment half of synthesize: every variable of one partition computed on the
 *                         GPU from the vanilla proof's openings (the instance slots below).
 *   mi_stacked_public_inputs <- generate_public_inputs (circuit/proof.hpp:186-269).
 * Instance slots (32 B each, Fr LE canonical, u64 indices in the low 8 bytes):
 *   0 replica_id, 1 comm_d, 2 comm_r, 3 comm_r_last, 4 comm_c; challenge c from 5 + c * stride:
 *   +0 challenge (u64), +1 data leaf, tree D siblings (leaf upward), tree R-last siblings, tree C siblings of
 *   the challenged column, then 6 DRG and 8 expander parents: index (u64), column (layers labels), tree C
 *   siblings.  Siblings of an arity-a level: the a - 1 other children in position order.
 * The layout is pinned by the reference's constraint counts (1,199,620 for 2 layers, 1 challenge, 8 nodes,
 * base 8; proof.cpp:137-155) and checked row for row against oracle/stacked_circuit.py. */
typedef struct {
    uint32_t layers, challenges;
    uint64_t nodes;
    uint32_t base_arity, sub_arity, top_arity, reserved;
} mi_stacked_shape;
typedef struct mi_stacked mi_stacked;
/* with_r1cs = 0 builds the witness program only (the R1CS stays with whoever built the key) */
int mi_stacked_build(const mi_stacked_shape *shape, int with_r1cs, mi_stacked **out);
/* out: constraints, inputs (with ONE), aux, instance slots, slots per challenge, tree D depth, siblings per
 * tree C / R-last path, program ops, program levels, SHA-256 blocks, Poseidon hashes, R1CS entries */
int mi_stacked_info(const mi_stacked *s, uint64_t out[12]);
/* the R1CS with 32-byte coefficients (materialised on the first call; pointers valid until mi_stacked_free):
 * the form mi_circuit_load and external tools take */
int mi_stacked_r1cs(const mi_stacked *s, mi_r1cs *out);
/* the circuit uploaded straight from the builder's compact form (column + coefficient-table index per entry,
 * 8 B instead of 36): mi_circuit_load without the host-side 32-byte coefficient arrays */
int mi_stacked_load(mi_ctx *ctx, const mi_stacked *s, mi_circuit **out);
/* (inputs - 1) x 32 B: the public inputs in generate_public_inputs order (without ONE) */
int mi_stacked_public_inputs(const mi_stacked *s, const uint8_t *slots, uint8_t *out);
/* z_dev: (inputs + aux) x 32 B on this context's GPU, fully written on return; slots refused if not canonical or
 * an index >= nodes (MI_ERR_ARG) */
int mi_stacked_witness_dev(mi_ctx *ctx, mi_stacked *s, const void *slots_dev, void *z_dev);
int mi_stacked_witness(mi_ctx *ctx, mi_stacked *s, const uint8_t *slots, uint8_t *z_out);
void mi_stacked_free(mi_stacked *s);
/* ---- Fallback PoSt circuit (Window / Winning PoSt; SURVEY.md 8(a) a2 + 8(f)#3) ------------------------------
 * Replaces the synthesis half of FallbackPoStCompound's circuit_proofs (the reference keeps the circuit's
 * data, post/fallback/circuit.hpp:38-86 Sector / FallbackPoStCircuit, and the vanilla side,
 * post/fallback/vanilla.hpp:188-251 prove_all_partitions, :398-411 generate_leaf_challenge; the synthesize
 * body is rust-fil-proofs storage-proofs-post fallback/circuit.rs): per sector comm_c, comm_r_last, comm_r
 * (public), Poseidon-2(comm_c, comm_r_last) == comm_r, and one private tree R-last inclusion proof per
 * challenge.  The same mi_stacked object and calls (info, r1cs, public_inputs, witness, free) serve it.
 * Instance slots: sector s from s * stride: +0 comm_r, +1 comm_c, +2 comm_r_last, then challenge n from
 * +3 + n * (2 + siblings): challenged leaf index (u64), leaf, tree R-last siblings (leaf upward, position
 * order).  Pinned by the reference's partition sizes (constants.hpp:85-89): 2349 sectors x 10 challenges at
 * 32 GiB (8-8-0 trees, 2^30 nodes) = 125,279,217 constraints; 2300 x 10 at 64 GiB (8-8-2, 2^31) = 129,887,900.
 * Public inputs: per sector comm_r, then the challenged leaf indices. */
typedef struct {
    uint32_t sectors, challenges; /* sectors per partition, challenges per sector */
    uint64_t nodes;               /* nodes per sector */
    uint32_t base_arity, sub_arity, top_arity, reserved;
} mi_post_shape;
int mi_post_build(const mi_post_shape *shape, int with_r1cs, mi_stacked **out);

/* R1CS satisfaction on the device: out[0] = rows with (A z)(B z) != (C z), out[1] = the first one (~0 if none) */
int mi_circuit_check_dev(mi_ctx *ctx, const mi_circuit *circuit, const void *z_dev, uint64_t out[2]);

/* ---- device timers (HIP events on the launching stream, resolved at existing sync points, so they
 * stay on inside timed regions).  out = 13 records x {ms, launches, units}:
 *   0 k_accum_level0<G1> (units = points)   1 k_accum_level0<G2>   2 whole G1 MSM   3 whole G2 MSM
 *   4 digits + sort + bucket bounds          5 NTT transforms (units = elements)   6 whole prove (units = constraints)
 *   7 witness H2D upload + canonical check on the copy stream (units = bytes)
 *   8 k_poseidon launches (units = hashes)  9 tree builders' label / data uploads (units = bytes)
 *  10 stacked witness phase A (units = ops)  11 phase B SHA-256 blocks (units = blocks)
 *  12 phase B Poseidon gadgets (units = hashes) */
int mi_ctx_get_stats(mi_ctx *ctx, double out[39]);
int mi_ctx_reset_stats(mi_ctx *ctx);
/* work counters since the last reset: out[0] / out[1] = mixed additions (non-zero signed digits)
 * issued by the G1 / G2 bucket accumulation -- the unit of the VALU roofline */
int mi_ctx_get_work(mi_ctx *ctx, uint64_t out[2]);
/* memory fallbacks since the last reset: out[0] = proofs, key generations and key loads that hit an
 * out-of-memory error and were re-run after the 2^128 split tables of the device's keys (the one being proven
 * first; keys in use by another context are left alone) and the context's idle scratch were released (a retried
 * proof takes the GLV split and is byte-identical; a second failure is returned as MI_ERR_INTERNAL), out[1] =
 * bytes released for them.
 * Replaces failing outright when several keys share one GPU, as GROTH_PARAM_MEMORY_CACHE keeps them
 * (libs/filecoin/include/nil/filecoin/proofs/caches.hpp:48-116). */
int mi_ctx_get_fallbacks(mi_ctx *ctx, uint64_t out[2]);
/* G1 (out[0]) and G2 (out[1]) MSMs run over a window table (mi_points_precompute, a small key's tables) since the
 * last reset */
int mi_ctx_get_table_msms(mi_ctx *ctx, uint64_t out[2]);
/* proofs since the last reset whose L and A MSMs ran over one shared plan (mi_srs_shared_la) */
int mi_ctx_get_shared_plans(mi_ctx *ctx, uint64_t *out);
/* proofs since the last reset whose A plan was derived from L's (keys below the shared plan's density rule: L's plan
 * carries A's density in its entries and A's plan is filtered out of it, without a digit pass or a sort of its own) */
int mi_ctx_get_derived_plans(mi_ctx *ctx, uint64_t *out);
/* TEST ONLY: the first attempt of each of the next `count` proofs on this context fails with a real out-of-memory
 * error after its NTT chain (count < 0: every proof until reset to 0), so the release-and-retry path runs at any
 * size.  Production code never calls it; nothing in the prove path reads the environment for it. */
int mi_ctx_inject_oom(mi_ctx *ctx, int64_t count);
/* TEST / BENCHMARK ONLY: process-wide A/B switches (csrc/tune.h lists them with their meaning: "msm_c", "msm_split",
 * "msm_glv", "msm_wt", "msm_wt_max_log", "msm_sort", "g2_l2", "prove_lanes", "prove_b1_lane", "tree_batch",
 * "sdr_prefetch", "plan_prio", "a_from_l", ...).  Every switch defaults to the measured production choice, and the library
 * reads no environment variable for them: a production prove runs the same windows, lanes and kernels whatever its
 * process environment holds.  mi_tune_set refuses an unknown name (MI_ERR_ARG); mi_tune_clear(name) restores one
 * default, mi_tune_clear(NULL) all of them; mi_tune_get reports whether a switch is set and its value.  No reference
 * counterpart (the reference has no GPU path to tune). */
int mi_tune_set(const char *name, int64_t value);
/* DEBUG BUILD ONLY (make fqcheck: -DMI_FQ_CHECK): violations of the device Fq magnitude invariant counted since load
 * (or the last reset) -- out[0] normalised values with |top limb| > 2^24, out[1] zero tests with |round(V / p)| > 3
 * (csrc/field.h).  A release build returns MI_ERR_ARG. */
int mi_fq_check_read(uint64_t out[2], int reset);
int mi_tune_clear(const char *name);
int mi_tune_get(const char *name, int64_t *value, int *is_set);
/* msm window size chosen for n points (exposed for tests / reports) */
unsigned mi_msm_window_bits(uint64_t n);

/* ---- Poseidon and the stacked-PoRep Merkle trees ---------------------------
 * Poseidon over Fr (BLS12-381 scalar field): state [2^arity - 1, x_1 .. x_arity], x^5, 8 full rounds and
 * 55 / 56 / 57 / 57 partial rounds for arity 2 / 4 / 8 / 11, Cauchy MDS 1 / (i + j + t), Grain-LFSR round
 * constants; digest = state[1].  Inputs must be canonical Fr (< r), MI_ERR_ARG otherwise.  Trees are
 * stored row by row, bottom-up (base row excluded), the layout of the reference's DiskTree / LCTree
 * stores.  Replaces:
 *   mi_poseidon_hash      <- crypto3::hash<crypto3::hashes::poseidon<FieldType, A, A>> as called by
 *                            hash_single_column (libs/storage/include/nil/filecoin/storage/proofs/porep/
 *                            stacked/vanilla/hash.hpp:37-47) and the tree hasher ([NOT IN TREE])
 *   mi_tree_c_build       <- generate_tree_c_gpu / ColumnTreeBuilder<ColumnArity, TreeArity>::
 *                            add_final_columns -> (base_data, tree_data)  (porep/stacked/vanilla/proof.hpp:
 *                            383-590; use_gpu_column_builder, core/configuration.hpp:51-56)
 *   mi_tree_r_last_build  <- generate_tree_r_last with use_gpu_tree_builder: encode(key, data) per node,
 *                            then TreeBuilder<Arity>::add_final_leaves -> tree_data of
 *                            get_merkle_tree_cache_size(leafs, arity, rows_to_discard) entries
 *                            (proof.hpp:630-760)
 *   mi_tree_build         <- TreeBuilder<Arity>::add_final_leaves over given leaves (same file)
 *   mi_tree_cache_size    <- get_merkle_tree_cache_size (merkletree; called at proof.hpp:717) */
/* (t, R_F, R_P) in shape; with non-null buffers also the (R_F + R_P) * t round constants and the t * t MDS
 * matrix, canonical 32-byte LE (tests / external checks) */
int mi_poseidon_constants(unsigned arity, uint8_t *round_constants, uint8_t *mds, uint32_t shape[3]);
/* digests[i] = Poseidon_arity(preimages[i * arity .. i * arity + arity - 1]) (32 B LE each) */
int mi_poseidon_hash(mi_ctx *ctx, unsigned arity, const uint8_t *preimages, uint64_t count, uint8_t *digests);
int mi_poseidon_hash_dev(mi_ctx *ctx, unsigned arity, const void *preimages_dev, uint64_t count, void *digests_dev);
/* entries of the cached rows: every row above the base except the rows_to_discard lowest of them */
int mi_tree_cache_size(uint64_t leaves, unsigned arity, unsigned rows_to_discard, uint64_t *out);
int mi_tree_build(mi_ctx *ctx, unsigned arity, const uint8_t *leaves, uint64_t leaf_count, unsigned rows_to_discard,
                  uint8_t *tree_out);
int mi_tree_build_dev(mi_ctx *ctx, unsigned arity, const void *leaves_dev, uint64_t leaf_count,
                      unsigned rows_to_discard, void *tree_dev);
/* tree C: column j = (layer_labels[0][j], .., layer_labels[layers - 1][j]) hashed with Poseidon_layers
 * (layers = 2 or 11 in Filecoin) into base_out[j]; tree_out = all rows above the base of the
 * tree_arity-ary Poseidon tree over them (mi_tree_cache_size(nodes, tree_arity, 0) entries).
 * Host variant: labels are streamed up in batches overlapped with the hashing.
 * Device variant: labels_dev is layer-major (layer l at entry l * nodes). */
int mi_tree_c_build(mi_ctx *ctx, unsigned layers, uint64_t nodes, const uint8_t *const *layer_labels,
                    unsigned tree_arity, uint8_t *base_out, uint8_t *tree_out);
int mi_tree_c_build_dev(mi_ctx *ctx, unsigned layers, uint64_t nodes, const void *labels_dev, unsigned tree_arity,
                        void *base_dev, void *tree_dev);
/* tree R-last: data[j] <- last_layer_labels[j] + data[j] (mod r: the replica, written back over data),
 * then the tree_arity-ary Poseidon tree over the replica; tree_out receives
 * mi_tree_cache_size(nodes, tree_arity, rows_to_discard) entries */
int mi_tree_r_last_build(mi_ctx *ctx, uint64_t nodes, const uint8_t *last_layer_labels, uint8_t *data,
                         unsigned tree_arity, unsigned rows_to_discard, uint8_t *tree_out);
int mi_tree_r_last_build_dev(mi_ctx *ctx, uint64_t nodes, const void *labels_dev, void *data_dev, unsigned tree_arity,
                             unsigned rows_to_discard, void *tree_dev);
/* inclusion proofs of count challenges (u64 leaf indices) in a device-resident tree: leaf_out[i] = leaves[c_i];
 * siblings_out[(i * H + j) * (arity - 1) ..] = the arity - 1 siblings of c_i's ancestor in row j (0 = leaves,
 * H = log_arity(leaf_count) rows), in position order skipping its own slot (that slot is digit j of c_i in
 * base arity).  tree_dev is the cached rows of mi_tree_build_dev / mi_tree_c_build_dev / mi_tree_r_last_build_dev
 * with the same rows_to_discard; discarded rows are rebuilt per challenge from the leaves WITH POSEIDON (trees C
 * and R-last; a SHA-256 tree D goes through mi_tree_d_inclusion_paths_dev, which never rebuilds).  Replaces
 * MerkleTree_gen_proof (tree D / tree C openings, porep/stacked/vanilla/proof.hpp:139-140, column_proof.hpp
 * make_proof) and MerkleTree_gen_cached_proof (tree R-last, proof.hpp:183-186).  A challenge >= leaf_count is
 * refused with MI_ERR_ARG before any read. */
int mi_tree_inclusion_paths_dev(mi_ctx *ctx, unsigned arity, const void *leaves_dev, uint64_t leaf_count,
                                unsigned rows_to_discard, const void *tree_dev, uint64_t count,
                                const void *challenges_dev, void *leaf_out_dev, void *siblings_out_dev);

/* ---- SDR labelling witness: SHA-256 labels of challenged nodes ------------------
 * label = SHA256(replica_id || u32_be(layer) || u64_be(node) || 0^20 || parent_0 .. parent_36) with byte 31
 * &= 0x3f, the parents repeated cyclically to 37; no parents (node 0): the 64-byte prefix alone.  Replaces:
 *   mi_sdr_labels / _dev        <- LabelingProof create_label (porep/stacked/vanilla/detail/processing/naive/
 *                                  labelling_proof.hpp:46-60) and EncodingProof::create_key
 *                                  (vanilla/encoding_proof.hpp:42-53) over parents_data_full; n_parents
 *                                  labels per entry are repeated to 37 as vanilla/proof.hpp:233-237 does
 *   mi_sdr_labeling_proofs_dev  <- the per-challenge labelling-proof loop of prove_layers
 *                                  (vanilla/proof.hpp:190-255): base parents read from the challenged layer,
 *                                  expander parents from the layer below (layer 1: base parents only),
 *                                  parents_data_full optionally written out (37 x 32 B per challenge)
 * Device layouts: layers u32[count], nodes / challenges u64[count], parents 32 B x n_parents per entry,
 * parent_idx u32[count x (n_base + n_exp)], layer labels layer-major (layer l at entry (l-1) x nodes_per_layer).
 * Out-of-range layers or parent indices are refused with MI_ERR_ARG before any gather. */
int mi_sdr_labels(mi_ctx *ctx, const uint8_t replica_id[32], uint64_t count, const uint32_t *layers,
                  const uint64_t *nodes, const uint8_t *parents, unsigned n_parents, uint8_t *labels);
int mi_sdr_labels_dev(mi_ctx *ctx, const uint8_t replica_id[32], uint64_t count, const void *layers_dev,
                      const void *nodes_dev, const void *parents_dev, unsigned n_parents, void *labels_dev);
/* tree D (comm_d): the binary SHA-256 tree over the sector's 32-byte data nodes, node = SHA256(left || right)
 * with byte 31 &= 0x3f (Sha256Hasher, truncated into Fr); tree_dev receives every row above the leaves,
 * bottom-up, leaf_count - 1 entries (mi_tree_cache_size(leaf_count, 2, 0)).  leaf_count a power of two.
 * Openings: mi_tree_d_inclusion_paths_dev (the layouts of mi_tree_inclusion_paths_dev at arity 2, every row
 * cached).  Replaces the tree D build of transform_and_replicate_layers / MerkleTree_gen_proof(tree_d)
 * (porep/stacked/vanilla/proof.hpp:139-140).  The SDR and tree _dev calls return with their outputs written. */
int mi_tree_d_build_dev(mi_ctx *ctx, const void *leaves_dev, uint64_t leaf_count, void *tree_dev);
int mi_tree_d_inclusion_paths_dev(mi_ctx *ctx, const void *leaves_dev, uint64_t leaf_count, const void *tree_dev,
                                  uint64_t count, const void *challenges_dev, void *leaf_out_dev,
                                  void *siblings_out_dev);
int mi_sdr_labeling_proofs_dev(mi_ctx *ctx, const uint8_t replica_id[32], unsigned n_layers,
                               uint64_t nodes_per_layer, const void *layer_labels_dev, uint64_t count,
                               const void *layers_dev, const void *challenges_dev, const void *parent_idx_dev,
                               unsigned n_base, unsigned n_exp, void *labels_dev, void *parents_out_dev);

#ifdef __cplusplus
}
#endif
#endif /* MI355X_GROTH16_H */
