// msm_g2.hip -- G2 (Fq2) instantiation of the Pippenger MSM (msm_impl.h).
#ifdef MI_G2_RED_UNCAPPED
#define MI_WAVES_RED  // A/B: the G2 reduction kernels without the two-wave register cap
#endif
#include "msm_impl.h"

namespace mi {

void msm_g2(Ctx &c, const g2_affine_t *bases, const fr_t *scalars, const uint32_t *idx, uint64_t n,
            g2_xyzz_t *result_host, const WinTable *wt, uint64_t wt_lo) {
    if (wt && wt->p && n && tune::get(tune::MSM_WT, 1) != 0) {  // tune::MSM_WT = 0: ignore the window tables
        msm_run_wt<fq2_t>(c, *wt, wt_lo, scalars, idx, n, result_host, wt->sparse);
        return;
    }
    msm_run<fq2_t>(c, bases, scalars, idx, n, result_host);
}

void msm_g2_planned(Ctx &c, const MsmPlan &plan, const g2_affine_t *bases, g2_xyzz_t *result_host) {
    if (!plan.total) {
        *result_host = g2_xyzz_t::inf();
        return;
    }
    ScopedTimer whole(c, &c.stats.msm_g2, plan.n);  // scalar-side phase timed by msm_prepare's caller
    msm_accumulate_impl<fq2_t>(c, plan, bases, result_host);
}

}  // namespace mi
