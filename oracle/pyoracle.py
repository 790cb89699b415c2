"""ctypes loader for the CPU oracle (oracle/hhmm_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker or the timed CPU baseline.  It
uses the product's request builder (hhmm_amd.api.PreparedRequest) so both
sides see byte-identical inputs, and returns results in the same layout.
"""
import ctypes as C
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent
REPO = ROOT.parent
sys.path.insert(0, str(REPO / "gsoc17-hhmm_amd"))

from hhmm_amd import _abi  # noqa: E402
from hhmm_amd.api import PreparedRequest  # noqa: E402

_LIBS = {}


def build():
    subprocess.run(["make", "-s", "-C", str(ROOT)], check=True)


def load(variant="cr"):
    """variant 'cr': correctly rounded log (the checker); 'libm': host libm log."""
    if variant in _LIBS:
        return _LIBS[variant]
    name = {"cr": "liboracle.so", "libm": "liboracle_libm.so"}[variant]
    if os.environ.get("HHMM_ORACLE_SAN") == "1":  # the ASan + UBSan build (tools/sanitize.sh)
        name = name.replace(".so", "_san.so")
        path = ROOT / "build" / name
        if not path.exists():
            subprocess.run(["make", "-s", "-C", str(ROOT), "sanitize"], check=True)
    path = ROOT / "build" / name
    if not path.exists():
        build()
    lib = C.CDLL(str(path))
    RP = C.POINTER(_abi.Request)
    SP = C.POINTER(_abi.Result)
    lib.hhmm_oracle_run.argtypes = [RP, SP, C.c_int]
    lib.hhmm_oracle_run.restype = C.c_int
    lib.hhmm_oracle_run_range.argtypes = [RP, SP, C.c_int64, C.c_int64, C.c_int]
    lib.hhmm_oracle_run_range.restype = C.c_int
    lib.hhmm_oracle_log_array.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int64]
    lib.hhmm_oracle_variant.restype = C.c_char_p
    _LIBS[variant] = lib
    return lib


def gqs(model, data, draws, pars=None, pairing="grid", nthreads=1, variant="cr", return_status=False,
        pair_range=None, uniforms=None, hat_rand=None):
    """Same contract as hhmm_amd.gqs, computed by the scalar CPU oracle."""
    lib = load(variant)
    pr = PreparedRequest(model, data, draws, pars, pairing, uniforms=uniforms, hat_rand=hat_rand)
    if pair_range is None:
        st = lib.hhmm_oracle_run(C.byref(pr.req), C.byref(pr.res), nthreads)
    else:
        st = lib.hhmm_oracle_run_range(C.byref(pr.req), C.byref(pr.res), pair_range[0], pair_range[1],
                                       nthreads)
    if st < 0:
        raise RuntimeError(f"oracle rejected the request ({st})")
    out = dict(pr.out)
    if return_status:
        out["pair_status"] = pr.status
        out["status"] = st
    return out


def exp_array(x, variant="cr"):
    import numpy as np
    lib = load(variant)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    lib.hhmm_oracle_exp_array(x.ctypes.data_as(C.POINTER(C.c_double)),
                              y.ctypes.data_as(C.POINTER(C.c_double)), x.size)
    return y


def det_array(which, x):
    """The FFBS contract's deterministic exp / log (which = "exp" / "log")."""
    import numpy as np
    lib = load("cr")
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    fn = lib.hhmm_oracle_det_exp_array if which == "exp" else lib.hhmm_oracle_det_log_array
    fn(x.ctypes.data_as(C.POINTER(C.c_double)), y.ctypes.data_as(C.POINTER(C.c_double)), C.c_int64(x.size))
    return y


def crmath_quick_check(which, x, ziv=False):
    """(max relative quick-vs-accurate distance, rounding-test fallbacks,
    mismatches, arguments covered) of hhmm_crmath.h's quick phase; which is
    "log" or "exp".  ziv=True appends (the device's one-fma test hhmm_round_ziv:
    fallbacks, accepted-but-not-correctly-rounded arguments -- must be 0)."""
    import numpy as np
    lib = load("cr")
    x = np.ascontiguousarray(x, dtype=np.float64)
    st = np.zeros(6)
    lib.hhmm_oracle_crmath_quick_check(C.c_int({"log": 0, "exp": 1}[which]),
                                       x.ctypes.data_as(C.POINTER(C.c_double)), C.c_int64(x.size),
                                       st.ctypes.data_as(C.POINTER(C.c_double)))
    out = (float(st[0]), int(st[1]), int(st[2]), int(st[3]))
    return out + (int(st[4]), int(st[5])) if ziv else out


def log_array(x, variant="cr"):
    import numpy as np
    lib = load(variant)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    lib.hhmm_oracle_log_array(x.ctypes.data_as(C.POINTER(C.c_double)),
                              y.ctypes.data_as(C.POINTER(C.c_double)), x.size)
    return y


LEG_FIELDS = {"price": "f64", "start": "i32", "end": "i32", "size_av": "f64", "f0": "i32", "f1": "i32",
              "f2": "i32", "feature": "i32", "trend": "i32", "x": "i32", "sign": "i32"}


def extract_features(price, size, time, alpha=0.25, variant="cr"):
    """Sequential oracle of tayal2009/R/feature-extraction.R:8-133 -> dict of leg columns."""
    import numpy as np
    from hhmm_amd import features as F
    lib = load(variant)
    lib.hhmm_oracle_extract_features.argtypes = [C.POINTER(F.Ticks), C.POINTER(F.Legs)]
    lib.hhmm_oracle_extract_features.restype = C.c_int
    tk, keep = F.make_ticks(price, size, time, alpha)
    n = tk.n
    legs, out = F.make_legs(n)
    st = lib.hhmm_oracle_extract_features(C.byref(tk), C.byref(legs))
    if st != 0:
        raise RuntimeError(f"oracle extract_features status {st} (legs {legs.n_legs})")
    m = legs.n_legs
    return {k: v[:m].copy() for k, v in out.items()}


def neighbouring_forecast(x, oblik_t, h=1, threshold=0.05):
    """Sequential oracle of hassan2005/R/forecast.R:1-31 (long-double sums, libm exp)."""
    import numpy as np
    from hhmm_amd import forecast as Fc
    lib = load("libm")
    lib.hhmm_oracle_neighbouring_forecast.argtypes = [C.POINTER(Fc.ForecastRequest), C.c_void_p]
    lib.hhmm_oracle_neighbouring_forecast.restype = C.c_int
    req, _keep, P = Fc.make_request(x, oblik_t, h, threshold)
    out = np.empty(P)
    if lib.hhmm_oracle_neighbouring_forecast(C.byref(req), out.ctypes.data) != 0:
        raise RuntimeError("oracle rejected the forecast request")
    return out


def constrain_draws(model, theta, K, L=0, M=0, variant="cr"):
    """Oracle of the parameters-block constraining transforms (oracle/params_oracle.c)."""
    import numpy as np
    from hhmm_amd import params as Pm
    lib = load(variant)
    lib.hhmm_oracle_constrain.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int64, C.c_void_p,
                                          C.POINTER(Pm.ParamOut)]
    lib.hhmm_oracle_constrain.restype = C.c_int64
    th = np.asfortranarray(theta, dtype=np.float64)
    po, out = Pm.alloc_outputs(model, th.shape[0], K, L, M)
    n = lib.hhmm_oracle_constrain(_abi.MODELS[model], K, L, M, th.shape[0], th.ctypes.data, C.byref(po))
    if n != th.shape[1]:
        raise RuntimeError(f"oracle consumed {n} values per draw, theta has {th.shape[1]}")
    return out
