"""Host mirror of parameter-draw ingestion (include/hhmm_params.h).

rstan maps a point of the sampler's unconstrained space to the parameters
block with `constrain_pars(fit, upars)` (stanc's write_array reading the
block with `in__.simplex_constrain(K)` etc.).  `constrain_draws()` does that
for S draws at once on the gfx950 engine and returns the arrays in the shapes
`extract()` gives -- ready to pass as `draws` to hhmm_amd.gqs().
"""
import ctypes as C

import numpy as np

from . import _abi

FIELDS = ["p_1k", "A_ij", "phi_k", "mu_k", "sigma_k", "w_km", "b_km", "s_k", "lambda_kl", "mu_kl", "s_kl",
          "p_11", "A_row", "hypermu_k"]

# parameters each program declares (hmm/stan/hmm.stan:13-22, ...), with their extract() shapes
PARAMS = {
    "hmm": {"p_1k": "SK", "A_ij": "SKK", "mu_k": "SK", "sigma_k": "SK"},
    "hmm-multinom": {"p_1k": "SK", "A_ij": "SKK", "phi_k": "SKL"},
    "iohmm-reg": {"p_1k": "SK", "w_km": "SKM", "b_km": "SKM", "s_k": "SK"},
    "iohmm-mix": {"p_1k": "SK", "w_km": "SKM", "lambda_kl": "SKL", "mu_kl": "SKL", "s_kl": "SKL"},
    "hhmm-tayal2009": {"p_11": "S", "A_row": "S22", "phi_k": "SKL"},
}
PARAMS["hmm-multinom-semisup"] = PARAMS["hmm-multinom"]
PARAMS["iohmm-hmix"] = dict(PARAMS["iohmm-mix"], hypermu_k="SK")
PARAMS["iohmm-hmix-lite"] = dict(PARAMS["iohmm-mix"], hypermu_k="SK")
PARAMS["hhmm-tayal2009-lite"] = PARAMS["hhmm-tayal2009"]


class ParamOut(C.Structure):
    _fields_ = [(f, C.c_void_p) for f in FIELDS]


def declare(lib):
    lib.hhmm_num_unconstrained.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int]
    lib.hhmm_num_unconstrained.restype = C.c_int64
    lib.hhmm_constrain_draws.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int64, C.c_void_p,
                                         C.POINTER(ParamOut), C.c_int]
    lib.hhmm_constrain_draws.restype = C.c_int
    lib.hhmm_constrain_draws_device.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int64, C.c_void_p,
                                                C.POINTER(ParamOut), C.c_void_p]
    lib.hhmm_constrain_draws_device.restype = C.c_int
    return lib


def alloc_outputs(model, S, K, L=0, M=0):
    shapes = {"S": (S,), "SK": (S, K), "SKK": (S, K, K), "SKL": (S, K, L), "SKM": (S, K, M), "S22": (S, 2, 2)}
    out = {name: np.full(shapes[code], np.nan, order="F") for name, code in PARAMS[model].items()}
    po = ParamOut(*[out[f].ctypes.data if f in out else None for f in FIELDS])
    return po, out


def constrain_draws(model, theta, K, L=0, M=0, device=-1, lib=None):
    """theta: (S, n_unc) unconstrained draws (rstan's unconstrain_pars order) ->
    {parameter: array} in extract() shapes."""
    from .api import HHMMError, load_library
    lib = declare(lib or load_library())
    th = np.asfortranarray(theta, dtype=np.float64)
    S = th.shape[0]
    n = lib.hhmm_num_unconstrained(_abi.MODELS[model], K, L, M)
    if n < 0 or th.shape[1] != n:
        raise ValueError(f"{model} with K={K} L={L} M={M} takes {n} unconstrained values per draw, got {th.shape}")
    po, out = alloc_outputs(model, S, K, L, M)
    st = lib.hhmm_constrain_draws(_abi.MODELS[model], K, L, M, S, th.ctypes.data, C.byref(po), int(device))
    if st < 0:
        raise HHMMError(st, lib.hhmm_last_error().decode())
    return out
