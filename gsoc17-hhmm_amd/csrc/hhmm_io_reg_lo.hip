/* iohmm-reg/stan/iohmm-reg.stan, K = 1..4: instantiates the IOHMM kernel of hhmm_iohmm.h. */
#include "hhmm_iohmm.h"

namespace hhmm {

hhmm_status run_io_reg_lo(const DevArgs &a, hipStream_t st)
{
    return launch_io_range<IO_REG, 1, 4>(a, st);
}

} // namespace hhmm
