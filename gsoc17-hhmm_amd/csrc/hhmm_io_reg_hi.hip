/* iohmm-reg/stan/iohmm-reg.stan, K = 5..8: instantiates the IOHMM kernel of hhmm_iohmm.h. */
#include "hhmm_iohmm.h"

namespace hhmm {

hhmm_status run_io_reg_hi(const DevArgs &a, hipStream_t st)
{
    return launch_io_range<IO_REG, 5, 8>(a, st);
}

} // namespace hhmm
