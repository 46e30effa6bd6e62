// msm_g1.hip -- G1 instantiation of the Pippenger MSM (msm_impl.h) + window heuristic.
#define MI_WAVES2        // G1: compiler-chosen occupancy (msm_impl.h)
#define MI_ACC_PREFETCH 1  // measured same box: accumulation 125.5 -> 123.6 ms per 2^26 MSM (G2: +4.6%, off)
#include "msm_impl.h"

namespace mi {

unsigned msm_window_bits(uint64_t n) { return msm_window_bits_for(n, 256); }

unsigned msm_window_bits_for(uint64_t n, unsigned sbits, bool glv) {
    // minimise (mixed adds) + 1.4 x (bucket-reduction full adds) over c; split plans (129-bit scalars)
    // keep c >= 9 so their ceil(129 / c) windows fit the split digit kernel (MAXW_S = 16)
    const unsigned cmin = sbits < 256 ? 9 : 4;
    // tune::MSM_C forces the window size of every MSM (test only; clamped to [cmin, 22]) so the tests
    // can run the production windows (c = 20..22 at 2^26 / 2^27) on instances the oracle checks quickly
    if (const int64_t cf = tune::get(tune::MSM_C, 0); cf > 0)
        return (unsigned)(cf < (int64_t)cmin ? (int64_t)cmin : cf > 22 ? 22 : cf);
    unsigned best = cmin;
    double best_cost = 1e300;
    for (unsigned c = cmin; c <= 22; c++) {
        unsigned nwin = (sbits + c - 1) / c;
        // GLV plans add one full addition (+ one multiplication) per bucket in k_glv_merge
        const double per_bucket = glv ? 3.0 : 2.0;
        double cost = (double)n * nwin + 1.4 * per_bucket * nwin * (double)(1u << (c - 1)) + 64.0 * nwin * c;
        if (cost < best_cost) {
            best_cost = cost;
            best = c;
        }
    }
    return best;
}

bool msm_use_split(uint64_t n) {
    // tune::MSM_SPLIT: 0 off, 1 (default) above 2^20 points, 2 always (tests).  Up to 2^20 points the
    // plain plan sorts every window in one onesweep call while the split plan sorts window by window: same box,
    // the 2^20 G1 MSM 6.05 -> 5.39 ms unsplit, the Winning-PoSt proof (2^19-point MSMs) unchanged, the 2^21
    // proof 40.6 -> 41.4 ms if its 2^21 - 1-point H MSM went unsplit (tools/split_sweep.sh).
    // tune::MSM_SPLIT_MIN = k splits from 2^k points instead.
    const int64_t mode = tune::get(tune::MSM_SPLIT, 1);
    if (mode == 2) return true;
    if (mode != 1) return false;
    if (tune::is_set(tune::MSM_SPLIT_MIN)) {
        const int64_t lg = tune::get(tune::MSM_SPLIT_MIN, 0);
        return n >= (1ull << (lg < 0 ? 0 : lg > 40 ? 40 : lg));
    }
    return n > (1ull << 20);
}

int msm_glv_mode() {
    // tune::MSM_GLV (test only): unset = auto (the 2^128 table where the key has one, GLV otherwise),
    // 0 = never GLV, 1 = always GLV (and key load builds no tables)
    const int64_t v = tune::get(tune::MSM_GLV, tune::UNSET);
    return v == tune::UNSET ? 2 : v != 0 ? 1 : 0;
}

void msm_g1(Ctx &c, const g1_affine_t *bases, const fr_t *scalars, const uint32_t *idx, uint64_t n,
            g1_xyzz_t *result_host, const g1_affine_t *bases_hi, bool subgroup, const WinTable *wt, uint64_t wt_lo) {
    // tune::MSM_WT = 0 ignores the window tables (A/B, tests)
    if (wt && wt->p && n && tune::get(tune::MSM_WT, 1) != 0) {
        msm_run_wt<fq_t>(c, *wt, wt_lo, scalars, idx, n, result_host, wt->sparse);
        return;
    }
    msm_run<fq_t>(c, bases, scalars, idx, n, result_host, bases_hi, subgroup);
}

unsigned msm_wt_window_bits(uint64_t n) {
    if (const int64_t cf = tune::get(tune::MSM_WT_C, 0); cf > 0) return (unsigned)(cf < 8 ? 8 : cf > 22 ? 22 : cf);
    // One bucket set for every window.  Per entry (n ceil(256 / c) of them): a mixed add (1 / 6.6e9 s, measured at
    // 2^20) and its sort (~0.03 ns); per bucket: the first reduction level's two full adds (~3e9 / s); plus the
    // latency-bound bit-row tree (~0.4 ms).  The top window of a 255-bit scalar holds 255 - (nwin - 1) c bits: a c
    // that leaves it a few bits piles the entries of every point into its few buckets (deep chunk trees: measured
    // 5.0 ms at c = 18 against 3.9 at c = 20), so c needs >= 2^(log2 n - 8) top-window buckets.
    unsigned lg = 0;
    while ((1ull << lg) < n) lg++;
    unsigned best = 16;
    double best_cost = 1e300;
    for (unsigned c = 8; c <= 22; c++) {
        const unsigned nwin = (256 + c - 1) / c;
        const int top = 255 - (int)((nwin - 1) * c);
        if (top < (int)lg - 8 && top < (int)c - 1) continue;
        const double cost = (double)n * nwin * (1.0 / 6.6e9 + 0.03e-9) + 2.0 * (double)(1u << (c - 1)) / 3e9 + 0.4e-3;
        if (cost < best_cost) best_cost = cost, best = c;
    }
    return best;
}

bool msm_prepare(Ctx &c, const fr_t *scalars, const uint32_t *idx, uint64_t n, MsmPlan &plan, bool split) {
    return msm_prepare_impl(c, scalars, idx, n, plan, split);
}

bool msm_prepare_g1_shared(Ctx &c, const fr_t *scalars, uint64_t n, MsmPlan &plan) {
    const bool glv = msm_use_split(n) && msm_glv_mode() != 0;
    return msm_prepare_impl(c, scalars, nullptr, n, plan, false, glv);
}

bool msm_prepare_marked(Ctx &c, const fr_t *scalars, uint64_t n, MsmPlan &plan, bool glv, const uint32_t *amark) {
    return msm_prepare_impl(c, scalars, nullptr, n, plan, !glv, glv, amark);
}

bool msm_derive_plan(Ctx &c, const MsmPlan &src, const uint32_t *rank_bits, uint64_t nreal_dst, uint32_t dst_base,
                     MsmPlan &plan) {
    return msm_derive_plan_impl(c, src, rank_bits, nreal_dst, dst_base, plan);
}

void msm_g1_planned(Ctx &c, const MsmPlan &plan, const g1_affine_t *bases, g1_xyzz_t *result_host,
                    const g1_affine_t *bases_hi) {
    if (!plan.total) {
        *result_host = g1_xyzz_t::inf();
        return;
    }
    ScopedTimer whole(c, &c.stats.msm_g1, plan.nreal ? plan.nreal : plan.n);  // scalar-side phase timed by msm_prepare's caller
    msm_accumulate_impl<fq_t>(c, plan, bases, result_host, bases_hi);
}

}  // namespace mi
