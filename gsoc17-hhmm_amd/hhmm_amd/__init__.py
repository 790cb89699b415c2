"""hhmm_amd -- MI355X (gfx950) engine for the HMM-family hot path of
moon1910/gsoc17-hhmm: forward filter, backward pass, smoothed posteriors and
Viterbi decoding of the Stan programs in hmm/, iohmm-*/ and tayal2009/,
evaluated for many (series x posterior draw) pairs at once.

The compute lives in libhhmm.so (C ABI: include/hhmm.h).  This package is the
host-side mirror of the reference's rstan boundary (`gqs`, shaped like
rstan::extract()) plus the synthetic-data and multi-GPU helpers used by
bench.py.
"""
from . import _abi  # noqa: F401
from .api import HHMMError, PreparedRequest, gqs, load_library, reshape_pairs  # noqa: F401

__version__ = "0.1.0"
