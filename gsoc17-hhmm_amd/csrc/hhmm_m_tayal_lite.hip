/* tayal2009/stan/hhmm-tayal2009-lite.stan, K = 4..4: instantiates the HMM-family kernels of hhmm_hmm.h. */
#include "hhmm_hmm.h"

namespace hhmm {

hhmm_status run_tayal_lite(const DevArgs &a, const hhmm_request *req, const hhmm_result *res, hipStream_t st)
{
    return run_model_range<HHMM_MODEL_TAYAL_LITE, 4, 4>(a, req, res, st);
}

} // namespace hhmm
