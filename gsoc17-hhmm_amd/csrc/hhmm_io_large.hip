/* The IOHMM programs (iohmm-reg, iohmm-mix, iohmm-hmix, iohmm-hmix-lite) at
 * 8 < K <= 32: the state-parallel sweep of hhmm_lkio.h (SURVEY.md §8 A3-A5,
 * A6-A11 at large K). */
#include "hhmm_lkio.h"

namespace hhmm {

hhmm_status run_large_iohmm(const DevArgs &a, hipStream_t st)
{
    if (a.model == HHMM_MODEL_IOHMM_REG)
        return launch_lkio<IO_REG>(a, st);
    return launch_lkio<IO_MIX>(a, st);
}

} // namespace hhmm
