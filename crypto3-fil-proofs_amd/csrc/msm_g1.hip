// msm_g1.hip -- G1 instantiation of the Pippenger MSM (msm_impl.h) + window heuristic.
#define MI_WAVES2        // G1: compiler-chosen occupancy (msm_impl.h)
#define MI_ACC_PREFETCH 1  // measured same box: accumulation 125.5 -> 123.6 ms per 2^26 MSM (G2: +4.6%, off)
#include "msm_impl.h"

namespace mi {

unsigned msm_window_bits(uint64_t n) {
    // minimise (mixed adds) + 1.4 x (bucket-reduction full adds) over c
    unsigned best = 4;
    double best_cost = 1e300;
    for (unsigned c = 4; c <= 22; c++) {
        unsigned nwin = (256 + c - 1) / c;
        double cost = (double)n * nwin + 1.4 * 2.0 * nwin * (double)(1u << (c - 1)) + 64.0 * nwin * c;
        if (cost < best_cost) {
            best_cost = cost;
            best = c;
        }
    }
    return best;
}

void msm_g1(Ctx &c, const g1_affine_t *bases, const fr_t *scalars, const uint32_t *idx, uint64_t n,
            g1_xyzz_t *result_host) {
    msm_run<fq_t>(c, bases, scalars, idx, n, result_host);
}

bool msm_prepare(Ctx &c, const fr_t *scalars, const uint32_t *idx, uint64_t n, MsmPlan &plan) {
    return msm_prepare_impl(c, scalars, idx, n, plan);
}

void msm_g1_planned(Ctx &c, const MsmPlan &plan, const g1_affine_t *bases, g1_xyzz_t *result_host) {
    if (!plan.total) {
        *result_host = g1_xyzz_t::inf();
        return;
    }
    ScopedTimer whole(c, &c.stats.msm_g1, plan.n);  // scalar-side phase timed by msm_prepare's caller
    msm_accumulate_impl<fq_t>(c, plan, bases, result_host);
}

}  // namespace mi
