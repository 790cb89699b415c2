"""Host mirror of the reference's nearest-neighbour forecast.

The reference computes, after fitting iohmm-hmix(-lite),
    oblik_t <- extract(stan.fit, pars = 'oblik_t')[[1]]                 # hassan2005/main.R:94
    neighbouring_forecast(x = dataset$x.unscaled, oblik_t = oblik_t, h = 1, threshold = 0.05)
                                                                        # hassan2005/main.R:138
(hassan2005/R/forecast.R:1-31).  `neighbouring_forecast()` below is that call
on the gfx950 engine (include/hhmm_forecast.h), batched over series: x is
[T] or [N, T]; oblik_t is [S, T] or the engine's GRID-ordered [P, T]
(p = s + S*n).  No CPU fallback.
"""
import ctypes as C

import numpy as np


class ForecastRequest(C.Structure):
    _fields_ = [
        ("n_series", C.c_int64),
        ("n_draws", C.c_int64),
        ("T", C.c_int32),
        ("h", C.c_int32),
        ("threshold", C.c_double),
        ("x", C.c_void_p),
        ("oblik_t", C.c_void_p),
    ]


def declare(lib):
    lib.hhmm_neighbouring_forecast.argtypes = [C.POINTER(ForecastRequest), C.c_void_p, C.c_int]
    lib.hhmm_neighbouring_forecast.restype = C.c_int
    lib.hhmm_neighbouring_forecast_device.argtypes = [C.POINTER(ForecastRequest), C.c_void_p, C.c_void_p]
    lib.hhmm_neighbouring_forecast_device.restype = C.c_int
    return lib


def make_request(x, oblik_t, h=1, threshold=0.05):
    """(request, kept arrays, P) with R's argument checks (forecast.R:2-4)."""
    x = np.asarray(x, dtype=np.float64)
    ob = np.asarray(oblik_t, dtype=np.float64)
    if x.ndim == 1:
        x = x.reshape(1, -1)
    N, T = x.shape
    if ob.ndim != 2 or ob.shape[1] != T or ob.shape[0] % N:
        raise ValueError("The size of the observation vector and the width of the likelihood array must be equal.")
    S = ob.shape[0] // N
    xf = np.asfortranarray(x)
    of = np.asfortranarray(ob)
    req = ForecastRequest(N, S, T, int(h), float(threshold), xf.ctypes.data, of.ctypes.data)
    return req, (xf, of), N * S


def neighbouring_forecast(x, oblik_t, h=1, threshold=0.05, device=-1, lib=None):
    from .api import HHMMError, load_library
    lib = declare(lib or load_library())
    req, _keep, P = make_request(x, oblik_t, h, threshold)
    out = np.empty(P)
    st = lib.hhmm_neighbouring_forecast(C.byref(req), out.ctypes.data, int(device))
    if st < 0:
        raise HHMMError(st, lib.hhmm_last_error().decode())
    return out
