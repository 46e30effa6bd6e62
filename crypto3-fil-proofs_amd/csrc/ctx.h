// ctx.h -- per-device context shared by the NTT, MSM and prover translation units.
//
// One mi_ctx per GPU: owns the stream, the twiddle tables and a grow-only
// scratch arena, and is internally serialised by a mutex like the reference's
// GROTH_PARAM_MEMORY_CACHE mutexes (libs/filecoin/include/nil/filecoin/proofs/caches.hpp:48-54).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "curve.h"
#include "field.h"
#include "fr29.h"
#include "tune.h"

namespace mi {

struct hip_error : std::runtime_error {
    hipError_t code;
    hip_error(hipError_t c, const std::string &what) : std::runtime_error(what), code(c) {}
};

#define MI_HIP(call)                                                                              \
    do {                                                                                          \
        hipError_t _e = (call);                                                                   \
        if (_e != hipSuccess)                                                                     \
            throw ::mi::hip_error(_e, std::string(#call) + " failed: " + hipGetErrorString(_e) + \
                                          " at " + __FILE__ + ":" + std::to_string(__LINE__));    \
    } while (0)

// A device buffer that only grows (no hipMalloc inside the timed steady state).  A growth that fails leaves
// the buffer empty (p = nullptr, cap = 0) -- never a null pointer behind a stale capacity, which a later
// smaller request would hand to a kernel -- and throws the out-of-memory error (prover.hip retries on it).
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    void *get(size_t bytes) {
        if (bytes > cap) {
            release();
            const size_t want = bytes + bytes / 8;
            void *q = nullptr;
            hipError_t e = hipMalloc(&q, want);
            size_t got = want;
            if (e != hipSuccess) {  // the 1/8 growth slack is optional: try the exact size before giving up
                (void)hipGetLastError();
                q = nullptr;
                e = hipMalloc(&q, bytes);
                got = bytes;
            }
            if (e != hipSuccess) MI_HIP(e);
            p = q;
            cap = got;
        }
        return p;
    }
    template <class T>
    T *as(size_t count) {
        return (T *)get(count * sizeof(T));
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    ~DevBuf() { release(); }
};

// Page-locked host staging for the small device -> host readbacks of a lane (bucket counts, chunk totals, window
// sums).  A pageable destination makes HIP stage the copy and hold the host thread inside hipMemcpyAsync until
// the stream drains, and those staged copies serialise across threads: in a Winning-PoSt proof (four lanes) a
// lane's synchronisation stalled 2-4 ms behind another lane's pending copy (rocprofv3 HIP runtime trace,
// DESIGN §5).  Copies into this buffer are plain asynchronous DMA, waited for by the lane's own stream sync.
struct PinnedBuf {
    void *p = nullptr;
    size_t cap = 0;
    void *get(size_t bytes) {
        if (bytes > cap) {
            release();
            const size_t want = bytes < 65536 ? 65536 : bytes;
            MI_HIP(hipHostMalloc(&p, want, hipHostMallocDefault));
            cap = want;
        }
        return p;
    }
    template <class T>
    T *as(size_t count) {
        return (T *)get(count * sizeof(T));
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
    ~PinnedBuf() { release(); }
};

// Twiddle tables for every power-of-two domain up to 2^32 (bellman: Fr::ROOT_OF_UNITY with
// S = 32, multiplicative generator 7).  w^e for e < 2^32 = LO[e & 0xffff] * HI[e >> 16].
struct NttTables {
    fr_t *fw_lo = nullptr, *fw_hi = nullptr;  // powers of omega_{2^32}
    fr_t *iv_lo = nullptr, *iv_hi = nullptr;  // powers of omega_{2^32}^-1
    fr_t *g_lo = nullptr, *g_hi = nullptr;    // powers of the coset generator 7
    fr_t *gi_lo = nullptr, *gi_hi = nullptr;  // powers of 7^-1
    fr29_t *fw_1024 = nullptr, *iv_1024 = nullptr;  // omega_1024^j, j < 512 (in-tile twiddles, 29-bit limbs)
    fr29_t *lo29[4] = {nullptr, nullptr, nullptr, nullptr};  // fw, iv, g, gi LO / HI tables in 29-bit limbs
    fr29_t *hi29[4] = {nullptr, nullptr, nullptr, nullptr};  // (the NTT passes)
};

// Per-kernel-class device time from HIP events recorded on the launching stream.  Event pairs are
// resolved lazily at the next point where the host synchronises anyway, so the timers stay on in
// the timed region without adding synchronisation.
struct KStat {
    double ms = 0;
    uint64_t launches = 0;
    uint64_t units = 0;  // points (MSM) or elements (NTT) processed by the timed launches
};
struct Stats {
    KStat accum_g1, accum_g2;  // k_accum_level0 (the bucket-accumulation hot loop)
    KStat msm_g1, msm_g2;      // whole MSM (digits -> sort -> accumulate -> reduce)
    KStat sort;                // digit extraction + radix sort + bucket bounds
    KStat ntt;                 // NTT passes (all launches of one transform)
    KStat prove;               // whole Groth16 prove (device part through host assembly)
    KStat h2d;                 // witness upload + canonical check on the copy stream (units = bytes)
    KStat poseidon;            // k_poseidon launches (units = hashes)
    KStat tree_h2d;            // tree builders' label / data uploads (units = bytes)
    KStat wit_a;               // stacked witness phase A (levelled light ops + native hashes; units = ops)
    KStat wit_sha;             // stacked witness phase B, SHA-256 gadget blocks (units = blocks)
    KStat wit_pos;             // stacked witness phase B, Poseidon gadgets (units = hashes)
    uint64_t madds_g1 = 0, madds_g2 = 0;  // mixed additions issued by k_accum_level0 (non-zero digits)
    uint64_t oom_retries = 0;      // proofs re-run after an out-of-memory error (prover.hip groth16_sums)
    uint64_t oom_freed_bytes = 0;  // split tables + scratch released for those retries
    uint64_t wt_msms = 0, wt_msms_g2 = 0;  // G1 / G2 MSMs that ran over a window table (msm_run_wt)
    uint64_t shared_la = 0;                // proofs whose L and A MSMs ran over one shared plan (Srs::a_aux)
    uint64_t derived_a = 0;                // proofs whose A plan was derived from L's (msm_derive_plan)
    static constexpr int NK = 13;
    void merge(const Stats &o) {
        madds_g1 += o.madds_g1;
        wt_msms += o.wt_msms;
        wt_msms_g2 += o.wt_msms_g2;
        shared_la += o.shared_la;
        derived_a += o.derived_a;
        madds_g2 += o.madds_g2;
        KStat *d[] = {&accum_g1, &accum_g2, &msm_g1, &msm_g2, &sort, &ntt, &prove, &h2d, &poseidon, &tree_h2d,
                      &wit_a, &wit_sha, &wit_pos};
        const KStat *x[] = {&o.accum_g1, &o.accum_g2, &o.msm_g1, &o.msm_g2, &o.sort, &o.ntt, &o.prove, &o.h2d,
                            &o.poseidon, &o.tree_h2d, &o.wit_a, &o.wit_sha, &o.wit_pos};
        for (int i = 0; i < NK; i++) {
            d[i]->ms += x[i]->ms;
            d[i]->launches += x[i]->launches;
            d[i]->units += x[i]->units;
        }
    }
};

struct Ctx;
struct EventTimer {
    struct Pending {
        hipEvent_t a, b;
        KStat *dst;
        uint64_t units;
    };
    std::vector<hipEvent_t> pool;
    std::vector<Pending> pending;
    hipEvent_t get() {
        if (pool.empty()) {
            hipEvent_t e;
            MI_HIP(hipEventCreate(&e));
            return e;
        }
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    // resolve every pending pair whose end event has completed (call after a stream sync)
    void resolve() {
        std::vector<Pending> keep;
        for (auto &p : pending) {
            if (hipEventQuery(p.b) != hipSuccess) {
                keep.push_back(p);
                continue;
            }
            float ms = 0;
            hipEventElapsedTime(&ms, p.a, p.b);
            p.dst->ms += ms;
            p.dst->launches += 1;
            p.dst->units += p.units;
            pool.push_back(p.a);
            pool.push_back(p.b);
        }
        pending.swap(keep);
    }
    ~EventTimer() {
        for (auto &p : pending) {
            hipEventDestroy(p.a);
            hipEventDestroy(p.b);
        }
        for (auto e : pool) hipEventDestroy(e);
    }
};

inline uint64_t next_ctx_uid() {
    static std::atomic<uint64_t> n{1};
    return n.fetch_add(1);
}

struct Ctx {
    const uint64_t uid = next_ctx_uid();  // never reused: keys per-context device state held by shared objects
    int device = 0;
    hipStream_t stream = nullptr;
    std::recursive_mutex mu;
    NttTables tw;
    DevBuf scratch[34];  // 0-19: MSM / NTT / upload temporaries (18-19: G2 second level), 20: prover vectors,
                         // 21-22: witness slots (capi.hip uploader; 21 also building-block inputs),
                         // 24-25: an MSM plan's multi-chunk bucket list and first chunk-tree level (msm_impl.h),
                         // 26-33: a derived plan's arrays (msm_derive_plan: they outlive the next msm_prepare)
    Stats stats;
    EventTimer timer;
    PinnedBuf pin;  // small readbacks (msm_impl.h); one lane's, reused call after call
    // test hook (mi_ctx_inject_oom): the next inject_oom proofs' first attempts fail with a real out-of-memory
    // error after the NTT chain (-1: every proof), exercising the release-and-retry path of groth16_sums
    int64_t inject_oom = 0;
    // Auxiliary lane: a second stream with its own scratch arena and timers, driven from a second
    // host thread inside one prove so MSMs that do not depend on the NTT chain overlap it (the
    // accumulation is VALU-bound, the NTT / sort phases are LDS- / HBM-bound).  Created on first
    // use; ctx_aux_free releases it.  An auxiliary lane's own `aux` is the next lane (small proofs run three).
    Ctx *aux = nullptr;
    hipStream_t aux_streams[2] = {nullptr, nullptr};  // (in the aux ctx) normal, high priority
    // tune::PLAN_PRIO: this lane's MSM plans on a high-priority stream (created on first use, PlanStream in
    // msm_impl.h), ordered after and before the lane's stream by two events
    hipStream_t plan_stream = nullptr;
    hipEvent_t plan_ev[2] = {nullptr, nullptr};
};

// the owner's auxiliary lane, its stream matched to the owner's current stream priority
Ctx &ctx_aux(Ctx &c);
void ctx_aux_free(Ctx &c);

// Records a start event now and an end event at scope exit, on the ctx stream; no synchronisation.
struct ScopedTimer {
    Ctx &c;
    KStat *dst;
    uint64_t units;
    hipEvent_t a;
    ScopedTimer(Ctx &ctx, KStat *s, uint64_t u = 0) : c(ctx), dst(s), units(u) {
        a = c.timer.get();
        MI_HIP(hipEventRecord(a, c.stream));
    }
    ~ScopedTimer() {  // must not throw: runs during stack unwinding too
        hipEvent_t b = nullptr;
        if (!c.timer.pool.empty()) {
            b = c.timer.pool.back();
            c.timer.pool.pop_back();
        } else if (hipEventCreate(&b) != hipSuccess) {
            return;
        }
        if (hipEventRecord(b, c.stream) != hipSuccess) return;
        c.timer.pending.push_back({a, b, dst, units});
    }
};

// Opt-in launch checking (tune debug_sync=1, tests only): synchronise after each launch and name the kernel
// that faulted.  Off by default (no synchronisation in the hot path).
void debug_sync(Ctx &c, const char *what);
#define MI_LAUNCHED(ctx, name)          \
    do {                                \
        MI_HIP(hipGetLastError());      \
        ::mi::debug_sync((ctx), (name)); \
    } while (0)

// ---- NTT (ntt.hip) ----
void ntt_init_tables(Ctx &c);
void ntt_free_tables(Ctx &c);
// DIF: natural order in -> bit-reversed out (forward uses omega, inverse omega^-1, no 1/n)
void ntt_dif(Ctx &c, fr_t *d, unsigned log_n, bool inverse);
// DIT: bit-reversed in -> natural out
void ntt_dit(Ctx &c, fr_t *d, unsigned log_n, bool inverse);
void bitrev_permute(Ctx &c, fr_t *d, unsigned log_n);
// DIF NTT whose last pass also multiplies position pos by g^(+-bitrev(pos)) * scale (and optionally
// converts to canonical): iNTT + coset shift (+ 1/d) in the same HBM passes
// iNTT -> coset shift * scale -> NTT in natural order (a, b, c of the QAP), one pass fewer than the
// two transforms separately
void ntt_coset_roundtrip(Ctx &c, fr_t *d, unsigned log_n, const fr_t &scale);
// The QAP tail with a and b already through ntt_coset_roundtrip: cc's coset roundtrip whose last pass also
// forms h = (a b - cc) zinv and runs the first pass of h's inverse coset transform, then the rest of that
// transform with scale and the canonical epilogue: a <- H (bit-reversed, canonical), cc clobbered.
// Returns false (nothing launched) when the domain takes a single pass (log_n <= 10).
bool ntt_coset_qap(Ctx &c, fr_t *a, const fr_t *b, fr_t *cc, unsigned log_n, const fr_t &scale, const fr_t &zinv);
void ntt_dif_coset_epilogue(Ctx &c, fr_t *d, unsigned log_n, bool inverse, bool inverse_gen, const fr_t &scale,
                            bool to_canonical);
// d[pos] *= g^(±bitrev(pos)) * scale (scale may be null)
void coset_scale_bitrev(Ctx &c, fr_t *d, unsigned log_n, bool inverse_gen, const fr_t *scale_host,
                        bool to_canonical);
void coset_scale_natural(Ctx &c, fr_t *d, unsigned log_n, bool inverse_gen, const fr_t *scale_host);
void scale_all(Ctx &c, fr_t *d, uint64_t n, const fr_t &s);
void fr_to_mont_inplace(Ctx &c, fr_t *d, uint64_t n);
void fr_from_mont_inplace(Ctx &c, fr_t *d, uint64_t n);

// ---- MSM (msm_impl.h, msm_g1.hip, msm_g2.hip) ----
// Scalar-side state of one MSM (digits sorted into buckets, chunked, chunk order): depends only on
// the scalars, so MSMs over the same scalars with different bases (B_G1 and B_G2 of one prove)
// share it.  Pointers are into the ctx scratch arena; valid until the next msm_prepare on the ctx.
constexpr unsigned MSM_PLAN_MAXW = 16;  // windows of a split plan (msm_impl.h MAXW_S)
struct MsmPlan {
    uint64_t n = 0;      // points of the plan (2 x the real points in split mode)
    uint64_t nreal = 0;  // split mode (non-zero): point j >= nreal is 2^128 * base[j - nreal], scalar halves
    unsigned cb = 0, nwin = 0;
    uint32_t nbk = 0, nb = 0, L0 = 0, maxcnt = 0, total = 0;
    uint64_t entries = 0;  // non-zero digits over all windows
    bool glv = false;      // split through the GLV endomorphism: nbk / nb count sub-buckets (2 per bucket)
    const uint32_t *vals_s = nullptr, *off = nullptr, *cnt = nullptr, *coff = nullptr, *ccnt = nullptr,
                   *chunk_bucket = nullptr, *order = nullptr;
    // buckets with more than one level-0 chunk (mlist[0, m)) and the first in-place tree level over them (per-bucket
    // partial counts qcnt / offsets qoff, l1_total partials), counted before the plan's one readback
    uint32_t m = 0, l1_total = 0, L1 = 16;
    uint32_t level_total[16] = {};  // partials of tree level l (msm_impl.h TREE_MAXL)
    uint32_t *mlist = nullptr, *qcnt = nullptr, *qoff = nullptr;
    // split plans: window w's entries are vals_s[w n, w n + wn[w]) (before the bucket bounds); marked: built with
    // A's density in its entries (msm_prepare_marked), so msm_derive_plan can filter it
    uint32_t wn[MSM_PLAN_MAXW] = {};
    bool marked = false;
};
// false when every scalar is zero (the MSM is the identity).  split: plan the 2n half-scalar points of
// the 2^128-shifted base table (msm_g1 with bases_hi); the plan then needs bases_hi too.
bool msm_prepare(Ctx &c, const fr_t *scalars, const uint32_t *idx, uint64_t n, MsmPlan &plan, bool split = false);
// the plan msm_g1 takes for subgroup bases without a 2^128 table: GLV split above the split threshold, plain below;
// one plan serves several G1 base sets over the same scalars (msm_g1_planned), e.g. L and the aux part of A
bool msm_prepare_g1_shared(Ctx &c, const fr_t *scalars, uint64_t n, MsmPlan &plan);
// L's plan over the aux witness z_aux (n scalars, split through the 2^128 tables or, glv, the endomorphism) with A's
// density marked in its entries (amark = Circuit::a_rank), then A's plan derived from it without a sort: the entries of
// variables with A density, in L's bucket order, their point indices moved to A's (dst_base + the variable's rank in
// rank_bits = Circuit::a_bits; the 2^128 / phi half at + nreal_dst).  The derived plan lives in scratch slots 26-33 of c (it survives the next msm_prepare on c,
// so L's accumulation can follow); false when it has no entry.
bool msm_prepare_marked(Ctx &c, const fr_t *scalars, uint64_t n, MsmPlan &plan, bool glv, const uint32_t *amark);
bool msm_derive_plan(Ctx &c, const MsmPlan &src, const uint32_t *rank_bits, uint64_t nreal_dst, uint32_t dst_base,
                     MsmPlan &plan);
void msm_g1_planned(Ctx &c, const MsmPlan &plan, const g1_affine_t *bases, g1_xyzz_t *result_host,
                    const g1_affine_t *bases_hi = nullptr);
void msm_g2_planned(Ctx &c, const MsmPlan &plan, const g2_affine_t *bases, g2_xyzz_t *result_host);
// Fixed-base window table of a G1 / G2 base set P_0 .. P_{stride-1}: p[w * stride + i] = 2^(c w) P_i for w < nwin =
// ceil(256 / c).  An MSM over it (msm_g1 with wt) puts every window's digits into ONE set of 2^(c - 1) buckets: the
// same mixed additions as a c-bit Pippenger, the bucket reduction of one window instead of nwin, and no window
// combination.  Memory: nwin x the base set.
struct WinTable {
    const void *p = nullptr;  // g1_affine_t or g2_affine_t
    uint64_t stride = 0;
    unsigned c = 0, nwin = 0;
    // the MSM's scalars are mostly zero digits (a witness vector): compact the entries before the sort
    bool sparse = false;
};
// window bits of the tables built for n-point base sets (MI_MSM_WT_C overrides; read per call)
unsigned msm_wt_window_bits(uint64_t n);
// builds the table of `n` bases into dst (nwin * n points); synchronises c's stream
void g1_window_table(Ctx &c, const g1_affine_t *bases, uint64_t n, unsigned wbits, g1_affine_t *dst);
void g2_window_table(Ctx &c, const g2_affine_t *bases, uint64_t n, unsigned wbits, g2_affine_t *dst);
// result = sum_i scalar[idx ? idx[i] : i] * bases[i]; scalars canonical (raw) Fr.
// bases_hi (optional): bases_hi[i] = 2^128 bases[i].  With it, large MSMs run in split mode: scalar
// k_i = lo_i + 2^128 hi_i becomes two 128-bit scalars over bases[i] and bases_hi[i], which halves the
// windows (and the bucket reduction) for the same number of mixed additions (MI_MSM_SPLIT: 0 off,
// 1 default above 2^20 points, 2 always).
// subgroup: every base is known to lie in the prime-order subgroup (a generated key, a checked load, or
// bases that passed mi_points_check_subgroup); only then may auto mode take the GLV split (glv.h).
// wt (optional): the window table of the base set `bases` belongs to, `bases` being its point wt_lo; the MSM then
// runs over the table (msm_run_wt) instead.
void msm_g1(Ctx &c, const g1_affine_t *bases, const fr_t *scalars, const uint32_t *idx, uint64_t n,
            g1_xyzz_t *result_host, const g1_affine_t *bases_hi = nullptr, bool subgroup = false,
            const WinTable *wt = nullptr, uint64_t wt_lo = 0);
// whether msm_g1 with a bases_hi table takes the split path for n points
bool msm_use_split(uint64_t n);
// G1 split mode through the GLV endomorphism (glv.h) instead of the 2^128 tables: MI_MSM_GLV unset -> 2
// (auto: GLV for subgroup-known bases without a table, e.g. a generated or checked key whose tables would
// not fit in HBM at key load), 0 -> never, 1 -> always (key load builds no tables; the caller asserts
// that every base is in the subgroup).  Same-box 2^26 proof: tables 525-526
// ms and 88.9 GB after setup, GLV 532-533 ms and 68.9 GB.
int msm_glv_mode();
// bases_hi table: out[i] = 2^128 in[i] (128 doublings, batch-normalised to affine); scratch slots 10, 11
void g1_shift128(Ctx &c, const g1_affine_t *in, uint64_t n, g1_affine_t *out);
void msm_g2(Ctx &c, const g2_affine_t *bases, const fr_t *scalars, const uint32_t *idx, uint64_t n,
            g2_xyzz_t *result_host,
            const WinTable *wt = nullptr, uint64_t wt_lo = 0);
// host-side window-size heuristic (exposed for tests)
unsigned msm_window_bits(uint64_t n);
// same for `n` points with scalars of `sbits` bits including the signed-digit carry (256 plain, 129 split)
unsigned msm_window_bits_for(uint64_t n, unsigned sbits, bool glv = false);

// ---- encodings (encode.hip) ----
// zcash uncompressed big-endian -> device Montgomery affine (zcash from_uncompressed flag rules).
// bad_dev[0] += malformed / non-canonical / off-curve points; with reject_inf, bad_dev[1] += infinities
void g1_decode_uncompressed(Ctx &c, const uint8_t *dev_bytes, g1_affine_t *out, uint64_t n, int *bad_dev,
                            bool reject_inf = false);
void g2_decode_uncompressed(Ctx &c, const uint8_t *dev_bytes, g2_affine_t *out, uint64_t n, int *bad_dev,
                            bool reject_inf = false);
// bad_dev[2] += points P with r P != O (the checked load's subgroup test)
void g1_subgroup_check(Ctx &c, const g1_affine_t *pts, uint64_t n, int *bad_dev);
void g2_subgroup_check(Ctx &c, const g2_affine_t *pts, uint64_t n, int *bad_dev);
// *bad_dev += entries >= r (witness validation: an Fr32 must represent a valid Fr, core/fr32.hpp:36-40)
void fr_count_noncanonical(Ctx &c, const fr_t *d, uint64_t n, int *bad_dev, hipStream_t st);
// device affine -> zcash uncompressed bytes (device buffer); perm_log != 0 un-bit-reverses the source
void g1_encode_uncompressed(Ctx &c, const g1_affine_t *in, uint8_t *dev_out, uint64_t n, unsigned perm_log,
                            uint64_t first = 0);
void g2_encode_uncompressed(Ctx &c, const g2_affine_t *in, uint8_t *dev_out, uint64_t n);
// canonical LE Fr bytes (already on device, 32B each) -> canonical, reduced mod r (in place)
void fr_canonicalize(Ctx &c, fr_t *d, uint64_t n);

}  // namespace mi
