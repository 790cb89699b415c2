/* hmm/stan/hmm.stan and hmm-multinom.stan at 8 < K <= 32: the state-parallel
 * kernels of hhmm_large.h, 16-lane groups up to K = 16 and
 * 32-lane groups above (24-state loops up to K = 24). */
#include "hhmm_lkscan.h"

namespace hhmm {

hhmm_status run_large(const DevArgs &a, hipStream_t st)
{
    /* 32-lane groups carry 24 or 32 states in their compile-time loops */
    if (a.model == HHMM_MODEL_HMM_GAUSS)
        return a.K <= 16 ? run_large_model<HHMM_MODEL_HMM_GAUSS, 16, 16>(a, st)
               : a.K <= 24 ? run_large_model<HHMM_MODEL_HMM_GAUSS, 32, 24>(a, st)
                           : run_large_model<HHMM_MODEL_HMM_GAUSS, 32, 32>(a, st);
    return a.K <= 16 ? run_large_model<HHMM_MODEL_HMM_MULTINOM, 16, 16>(a, st)
           : a.K <= 24 ? run_large_model<HHMM_MODEL_HMM_MULTINOM, 32, 24>(a, st)
                       : run_large_model<HHMM_MODEL_HMM_MULTINOM, 32, 32>(a, st);
}

} // namespace hhmm
