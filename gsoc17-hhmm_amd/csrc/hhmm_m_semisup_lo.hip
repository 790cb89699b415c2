/* hmm/stan/hmm-multinom-semisup.stan, K = 1..4: instantiates the HMM-family kernels of hhmm_hmm.h. */
#include "hhmm_hmm.h"

namespace hhmm {

hhmm_status run_semisup_lo(const DevArgs &a, const hhmm_request *req, const hhmm_result *res, hipStream_t st)
{
    return run_model_range<HHMM_MODEL_HMM_MULTINOM_SEMISUP, 1, 4>(a, req, res, st);
}

} // namespace hhmm
