// tune.h -- test / benchmark A/B switches of the library (TEST ONLY; mi_tune_set in the C ABI).
//
// Every switch defaults to the measured production choice.  Nothing in the library reads the environment for
// them: a production prove runs the same window sizes, lanes and kernels whatever variables its process carries.
// Tests and the benchmark's A/B legs set them through mi_tune_set / mi_tune_clear (process-wide, atomic; a value
// set while proofs run takes effect at the next MSM / prove / tree call that reads it).
#pragma once
#include <atomic>
#include <climits>
#include <cstdint>
#include <cstring>

namespace mi::tune {

enum Knob : int {
    MSM_C = 0,         // window bits of every plain / split MSM (clamped to [cmin, 22])
    MSM_SPLIT,         // 0 off, 1 (default) above 2^20 points (or from 2^MSM_SPLIT_MIN), 2 always
    MSM_SPLIT_MIN,     // split from 2^k points instead of above 2^20
    MSM_GLV,           // unset: auto (tables where the key has them, GLV otherwise); 0 never, 1 always
    MSM_WT,            // 0: ignore the keys' window tables
    MSM_WT_C,          // window bits of a window table (clamped to [8, 22])
    MSM_WT_MAX_LOG,    // keys with a domain <= 2^k build window tables (default 21; 0 = never)
    MSM_L0,            // sorted entries per level-0 chunk (default 64, 128 for plans of >= 2^24 points a window)
    MSM_L1,            // chunk partials per tree-level thread (power of two, default 16)
    MSM_SORT,          // 1: the per-window sorted path (and digit compaction) at any size
    MSM_BITSUM,        // 0: one-window plans reduce through the running-sum kernels
    MSM_SEGA_LOG,      // first-level bucket-reduction segments 2^k
    MSM_SEGB_LOG,      // second-level segments 2^k (<= 2^13)
    MSM_BS_SEG_LOG,    // bit-row reduction: first-level segments >= 2^k (default 16)
    MSM_BS_G0,         // bit-row reduction: items per thread of k_bitsum_first
    G2_L2,             // 0 off, 1 (default) from 2^20 level-1 buckets, 2 always: G2 reduction as a second-level MSM
    G2_AFF_K,          // buckets per batch inversion of k_bucket_affine (32 / 64 / 128, default 64)
    QAP_FUSED,         // 0: the separate A B - C division pass
    PROVE_LANES,       // 1: one lane (the auxiliary lane's MSMs after the main lane on the same stream)
    PROVE_WIDE_LOG,    // proofs with domain <= 2^k run three auxiliary lanes (default 21)
    PROVE_B1_LANE,     // small proofs: B_G1 after A (2, default), after L (1), beside B_G2 (0)
    AUX_ORDER,         // 1: L before B on the auxiliary lane
    LANE_PRIO,         // 1: auxiliary lane above a normal main lane, 2: normal under a high-priority main lane
    WIT_POS_LANES,     // largest Poseidon witness launch on 16-lane hashes (default 65536; 0 never)
    SDR_PREFETCH,      // 1: software-pipelined parent gathers
    POSEIDON_PAIR,     // 1 wave-pair kernel, 0 one thread per hash (default: pairs for arity 8, 11)
    TREE_BATCH,        // columns / leaves per upload batch of the host tree builders (default 2^21)
    DEBUG_SYNC,        // 1: synchronise and report after every debug_sync point
    PLAN_PRIO,         // 1: MSM plans (digits, sort, bounds, chunking) on a high-priority stream of their lane
    A_FROM_L,          // 0: A's plan sorted on its own instead of derived from L's (below the shared-plan density)
    NKNOBS
};

constexpr int64_t UNSET = INT64_MIN;

inline constexpr const char *kNames[NKNOBS] = {
    "msm_c",          "msm_split",      "msm_split_min",  "msm_glv",       "msm_wt",         "msm_wt_c",
    "msm_wt_max_log", "msm_l0",         "msm_l1",         "msm_sort",      "msm_bitsum",     "msm_sega_log",
    "msm_segb_log",   "msm_bs_seg_log", "msm_bs_g0",      "g2_l2",         "g2_aff_k",       "qap_fused",
    "prove_lanes",    "prove_wide_log", "prove_b1_lane",  "aux_order",     "lane_prio",      "wit_pos_lanes",
    "sdr_prefetch",   "poseidon_pair",  "tree_batch",     "debug_sync",    "plan_prio",
    "a_from_l"};

inline std::atomic<int64_t> g_knobs[NKNOBS] = {};  // zero-initialised; reset() / first use mark them UNSET
inline std::atomic<bool> g_init{false};

inline void reset() {
    for (int k = 0; k < NKNOBS; k++) g_knobs[k].store(UNSET, std::memory_order_relaxed);
    g_init.store(true, std::memory_order_release);
}

inline int find(const char *name) {
    if (!name) return -1;
    for (int k = 0; k < NKNOBS; k++)
        if (strcmp(kNames[k], name) == 0) return k;
    return -1;
}

// the knob's value, or dflt while it is unset
inline int64_t get(Knob k, int64_t dflt) {
    if (!g_init.load(std::memory_order_acquire)) return dflt;
    const int64_t v = g_knobs[k].load(std::memory_order_relaxed);
    return v == UNSET ? dflt : v;
}

inline bool is_set(Knob k) { return get(k, UNSET) != UNSET; }

inline void set(Knob k, int64_t v) {
    static const bool once = (reset(), true);
    (void)once;
    g_knobs[k].store(v, std::memory_order_relaxed);
}

}  // namespace mi::tune
