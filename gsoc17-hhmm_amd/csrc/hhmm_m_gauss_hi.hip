/* hmm/stan/hmm.stan, K = 5..8: instantiates the HMM-family kernels of hhmm_hmm.h. */
#include "hhmm_hmm.h"

namespace hhmm {

hhmm_status run_gauss_hi(const DevArgs &a, const hhmm_request *req, const hhmm_result *res, hipStream_t st)
{
    return run_model_range<HHMM_MODEL_HMM_GAUSS, 5, 8>(a, req, res, st);
}

} // namespace hhmm
