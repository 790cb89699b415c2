/* hmm/stan/hmm.stan and hmm-multinom.stan at 8 < K <= 32: the state-parallel
 * kernels of hhmm_large.h, 16-lane groups up to K = 16 and
 * 32-lane groups above. */
#include "hhmm_large.h"

namespace hhmm {

hhmm_status run_large(const DevArgs &a, hipStream_t st)
{
    if (a.model == HHMM_MODEL_HMM_GAUSS)
        return a.K <= 16 ? run_large_model<HHMM_MODEL_HMM_GAUSS, 16>(a, st)
                         : run_large_model<HHMM_MODEL_HMM_GAUSS, 32>(a, st);
    return a.K <= 16 ? run_large_model<HHMM_MODEL_HMM_MULTINOM, 16>(a, st)
                     : run_large_model<HHMM_MODEL_HMM_MULTINOM, 32>(a, st);
}

} // namespace hhmm
