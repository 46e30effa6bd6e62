// msm_g1.hip -- G1 instantiation of the Pippenger MSM (msm_impl.h) + window heuristic.
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

}  // namespace mi
