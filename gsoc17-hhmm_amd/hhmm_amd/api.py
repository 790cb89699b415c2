"""Host-side mirror of the reference's model boundary.

The reference evaluates one Stan program per fit:
    fit <- rstan::stan(file, data = list(T=..., K=..., x=...), ...)   # hmm/main.R:49-54
    alpha <- rstan::extract(fit, pars = 'alpha_tk')[[1]]               # hmm/main.R:67
and rstan's write_array recomputes the transformed parameters / generated
quantities for every saved draw.  `gqs()` below is that per-draw evaluation
for a whole batch: `data` is the Stan data block (batched over series),
`draws` is what extract() returns for the parameters block, and the result
is a dict of arrays shaped like extract(pars=...) -- [S, T, K] for one series,
[S, N, T, K] when N series are evaluated under the same S draws.

Arrays are numpy in Fortran order: the memory of an R array, so the same
buffers feed the C ABI (include/hhmm.h) without a copy.  The compute runs on
the gfx950 engine (libhhmm.so); there is no CPU fallback.
"""
import ctypes as C
import os
import pathlib

import numpy as np

from . import _abi

_PKG = pathlib.Path(__file__).resolve().parent
LIB_PATH = _PKG.parent / "lib" / "libhhmm.so"
_lib = None


class HHMMError(RuntimeError):
    def __init__(self, status, message):
        super().__init__(f"hhmm status {status}: {message}")
        self.status = status


def _init_torch_first():
    """PyTorch-ROCm ships its own HIP runtime next to the one libhhmm.so links
    (/opt/rocm).  Both work in one process only when torch's initialises the
    device first (measured on MI355X: the other order leaves torch with "No HIP
    GPUs are available"), so a process that has imported torch gets its device
    context before the engine's first HIP call."""
    import sys
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_available():
        torch.cuda.init()


def load_library(path=None):
    """Loads libhhmm.so; raises ImportError if it has not been built."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = pathlib.Path(path) if path else pathlib.Path(os.environ.get("HHMM_LIB", LIB_PATH))
    if not p.exists():
        raise ImportError(
            f"libhhmm.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the engine has no CPU fallback)")
    _init_torch_first()
    lib = _abi.declare(C.CDLL(str(p)))
    if path is None:
        _lib = lib
    return lib


def _f64(a):
    return np.asfortranarray(a, dtype=np.float64)


def _i32(a):
    return np.asfortranarray(a, dtype=np.int32)


# Which Stan data-block name feeds which ABI field, per model.
_REAL_X = {"hmm", "iohmm-reg", "iohmm-mix", "iohmm-hmix", "iohmm-hmix-lite"}


def _series_array(a, N, kind):
    a = np.asarray(a)
    if a.ndim == 1:  # one series: x[T]
        a = a.reshape(1, -1)
    if a.shape[0] != N:
        raise ValueError(f"expected {N} series, got array of shape {a.shape}")
    return _i32(a) if kind == "i32" else _f64(a)


class PreparedRequest:
    """A request plus the numpy buffers it points at (kept alive together)."""

    def __init__(self, model, data, draws, pars, pairing="grid", device=-1, uniforms=None, flags=0,
                 hat_rand=None):
        if model not in _abi.MODELS:
            raise ValueError(f"unknown model {model!r}; one of {sorted(_abi.MODELS)}")
        self.model = model
        self.keep = []
        req = _abi.Request()
        req.abi_version = _abi.ABI_VERSION
        req.model = _abi.MODELS[model]
        req.pairing = {"grid": _abi.PAIR_GRID, "zip": _abi.PAIR_ZIP, "block": _abi.PAIR_BLOCK}[pairing]
        req.device = device
        req.flags = int(flags)

        xkey = "x_t" if model.startswith("iohmm") else "x"
        x = np.asarray(data[xkey])
        N = 1 if x.ndim == 1 else x.shape[0]
        Tmax = x.shape[-1]
        d = req.data
        d.n_series = N
        d.T_max = Tmax
        d.K = int(data["K"])
        d.L = int(data.get("L", 0))
        d.M = int(data.get("M", 0))
        d.G = int(data.get("G", 0))
        if model in _REAL_X:
            d.x_real = self._ptr(_series_array(x, N, "f64"))
        else:
            d.x_int = self._ptr(_series_array(x, N, "i32"))
        if "T" in data and np.ndim(data["T"]) > 0:
            d.T = self._ptr(_i32(np.asarray(data["T"]).reshape(N)))
        if "g" in data:
            d.g = self._ptr(_series_array(data["g"], N, "i32"))
        if "sign" in data:
            d.sign = self._ptr(_series_array(data["sign"], N, "i32"))
        if "u_tm" in data:
            u = np.asarray(data["u_tm"], dtype=np.float64)
            if u.ndim == 2:  # one series: u_tm[T][M]
                u = u.reshape(1, *u.shape)
            d.u = self._ptr(_f64(u))
        if "x_oos" in data:
            xo = np.asarray(data["x_oos"])
            d.T_oos_max = xo.shape[-1]
            d.x_oos = self._ptr(_series_array(xo, N, "i32"))
            d.sign_oos = self._ptr(_series_array(data["sign_oos"], N, "i32"))
            if "T_oos" in data and np.ndim(data["T_oos"]) > 0:
                d.T_oos = self._ptr(_i32(np.asarray(data["T_oos"]).reshape(N)))
        if "hyperparams" in data:
            d.hyperparams = self._ptr(_f64(np.asarray(data["hyperparams"]).reshape(-1)))

        S = None
        for name in _abi.DRAW_ARRAYS:
            if name in draws:
                arr = _f64(draws[name])
                if arr.ndim == 0:
                    arr = arr.reshape(1)
                if S is None:
                    S = arr.shape[0]
                elif arr.shape[0] != S:
                    raise ValueError(f"draw array {name} has {arr.shape[0]} draws, expected {S}")
                setattr(req.draws, name, self._ptr(arr))
        if S is None:
            raise ValueError("no draw arrays given")
        req.draws.n_draws = S
        self.N, self.S, self.Tmax, self.K = N, S, Tmax, d.K
        self.T_oos_max = d.T_oos_max
        if pairing == "block" and S % N:
            raise ValueError(f"block pairing needs n_draws ({S}) to be a multiple of n_series ({N})")
        self.P = N * S if pairing == "grid" else (S if pairing == "block" else N)

        if pars is None:
            pars = ["loglik", "alpha_tk", "gamma_tk", "zstar_t", "logp_zstar"]
        self.pars = list(pars)
        req.outputs = 0
        res = _abi.Result()
        self.out = {}
        for name in self.pars:
            if name not in _abi.OUT:
                raise ValueError(f"unknown output {name!r}")
            req.outputs |= _abi.OUT[name]
            dt, shape = _abi.RESULT_ARRAYS[name]
            arr = self._alloc(dt, shape)
            self.out[name] = arr
            setattr(res, name, arr.ctypes.data)
        if "z_ffbs" in self.pars:
            if uniforms is None:
                raise ValueError("z_ffbs (FFBS) needs uniforms of shape (P, T_max)")
            uu = _f64(uniforms)
            if uu.shape != (self.P, Tmax):
                raise ValueError(f"uniforms must have shape {(self.P, Tmax)}, got {uu.shape}")
            req.ffbs_u = self._ptr(uu)
        if {"hatz_t", "hatl_t", "hatx_t"} & set(self.pars):
            if hat_rand is None:
                raise ValueError("hatz_t / hatl_t / hatx_t need hat_rand of shape (P, T_max, 3)")
            hr = _f64(hat_rand)
            if hr.shape != (self.P, Tmax, 3):
                raise ValueError(f"hat_rand must have shape {(self.P, Tmax, 3)}, got {hr.shape}")
            req.hat_rand = self._ptr(hr)
        self.status = np.zeros(self.P, dtype=np.int32)
        res.pair_status = self.status.ctypes.data
        self.req, self.res = req, res

    def _ptr(self, arr):
        self.keep.append(arr)
        return arr.ctypes.data

    def _alloc(self, dt, code):
        P, T, K, To = self.P, self.Tmax, self.K, self.T_oos_max
        Tz = To if self.model == "hhmm-tayal2009-lite" else T
        shape = {"P": (P,), "PTK": (P, T, K), "PT": (P, T), "PTz": (P, Tz), "PToK": (P, To, K)}[code]
        if dt == "f64":
            return np.full(shape, np.nan, dtype=np.float64, order="F")
        return np.zeros(shape, dtype=np.int32, order="F")


def gqs(model, data, draws, pars=None, pairing="grid", device=-1, lib=None, return_status=False, uniforms=None,
        flags=0, hat_rand=None):
    """Evaluates the model's TP/GQ outputs for every (series, draw) pair on the GPU.

    Returns {name: array} with pair-major shapes (P, T, K) / (P, T) / (P,);
    pair p = s + S*n under "grid" pairing (see reshape_pairs).  "z_ffbs" (a
    forward-filtering backward-sampling draw) consumes the
    caller's uniforms, shape (P, T_max), values in (0, 1).  `flags`: HHMM_FLAG_*
    (e.g. force / forbid the parallel scan over T, _abi.FLAG_SCAN_*).  The IOHMM
    fitted-output draws hatz_t / hatl_t / hatx_t (Stan's categorical_rng /
    normal_rng) consume `hat_rand`, shape (P, T_max, 3): a uniform for hatz, a
    uniform for hatl and a standard normal deviate for hatx per (pair, t)."""
    lib = lib or load_library()
    pr = PreparedRequest(model, data, draws, pars, pairing, device, uniforms, flags, hat_rand)
    st = lib.hhmm_run(C.byref(pr.req), C.byref(pr.res))
    if st < 0:
        raise HHMMError(st, lib.hhmm_last_error().decode())
    out = dict(pr.out)
    if return_status:
        out["pair_status"] = pr.status
        out["status"] = st
    return out


def reshape_pairs(arr, S, N):
    """(P, ...) -> (S, N, ...): rstan's [S, ...] slab per series (p = s + S*n)."""
    return arr.reshape((S, N) + arr.shape[1:], order="F")
