/* iohmm-mix/stan/iohmm-{mix,hmix,hmix-lite}.stan, K = 1..4: instantiates the IOHMM kernel of hhmm_iohmm.h. */
#include "hhmm_iohmm.h"

namespace hhmm {

hhmm_status run_io_mix_lo(const DevArgs &a, hipStream_t st)
{
    return launch_io_range<IO_MIX, 1, 4>(a, st);
}

} // namespace hhmm
