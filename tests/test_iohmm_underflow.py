"""CPU: the inputs of tests/test_gpu_iohmm_underflow.py do drive the IOHMM
linear-space filter below the sweeps' underflow check (2^-960), so the GPU
tests exercise the log-space re-run (hhmm_iolog.hip); the mild control case
does not.  The oracle stays finite on them, as the reference's log space does
(iohmm-reg/stan/iohmm-reg.stan:59-78)."""
import numpy as np
import pytest

from hhmm_amd import synth
from iohmm_linear import IO_WEAK, reg_linear_floor


@pytest.mark.parametrize("K,T,scale", [(4, 10_000, 400.0), (4, 10_000, 2000.0), (16, 120, 400.0), (16, 2000, 400.0)])
def test_saturated_transitions_underflow_the_linear_filter(oracle, K, T, scale):
    data, draws = synth.iohmm_reg(N=2, S=6, T=T, K=K, M=4)
    draws["w_km"] = draws["w_km"] * scale
    assert reg_linear_floor(data, draws) < IO_WEAK
    ref = oracle.gqs("iohmm-reg", data, draws, pars=["loglik"], nthreads=8)
    assert np.isfinite(ref["loglik"]).all()


def test_mild_transitions_stay_above_the_check():
    data, draws = synth.iohmm_reg(N=2, S=6, T=2000, K=4, M=4)
    assert reg_linear_floor(data, draws) > 1e-30
