// msm_g2.hip -- G2 (Fq2) instantiation of the Pippenger MSM (msm_impl.h).
#include "msm_impl.h"

namespace mi {

void msm_g2(Ctx &c, const g2_affine_t *bases, const fr_t *scalars, const uint32_t *idx, uint64_t n,
            g2_xyzz_t *result_host) {
    msm_run<fq2_t>(c, bases, scalars, idx, n, result_host);
}

}  // namespace mi
