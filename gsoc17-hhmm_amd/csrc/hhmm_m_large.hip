/* hmm/stan/hmm.stan and hmm-multinom.stan at 8 < K <= 32: the state-parallel
 * kernels of hhmm_large.h. */
#include "hhmm_large.h"

namespace hhmm {

hhmm_status run_large(const DevArgs &a, hipStream_t st)
{
    if (a.model == HHMM_MODEL_HMM_GAUSS)
        return run_large_model<HHMM_MODEL_HMM_GAUSS>(a, st);
    return run_large_model<HHMM_MODEL_HMM_MULTINOM>(a, st);
}

} // namespace hhmm
