"""One long series split over ranks along T ("single very long
series": each GPU scans its T-chunk, all-gathers the K x K chunk summaries and
fixes up its prefix).

The engine side is include/hhmm.h `hhmm_segment`: a rank's request holds the
steps [t0, t1) of every pair's series, and runs in two calls on one workspace:

  summary()  the window's T-scan chunk products and their ordered products per
             pair: SF (forward; the state entering the window times SF is the
             state leaving it), SQ (backward; SQ times beta leaving the window
             is beta entering it), their power-of-two exponents and the
             Gaussian log scale -- 2K^2 + 3 doubles per pair;
  finish()   given the state entering the window and beta leaving it: the
             scan's phases 2 and 3 for the window's steps (loglik on the last
             window only).

`boundaries()` chains the gathered summaries (host numpy, K x K per pair per
window).  `dist.gqs_tsplit` runs the whole exchange over torch.distributed;
the GPU tests run it window by window in one process and over two gloo ranks.
The reference evaluates every series sequentially inside one Stan program
(e.g. tayal2009/stan/hhmm-tayal2009.stan:46-128); the segments must give its
results within tests/tolerances.py.
"""
import ctypes as C

import numpy as np

from . import _abi, api

LN2 = float(np.log(2.0))
SEGMENT_OUTPUTS = ("loglik", "alpha_tk", "beta_tk", "ungamma_tk", "gamma_tk")


class Segment(C.Structure):
    _fields_ = [("first", C.c_int32), ("last", C.c_int32), ("summary", C.c_void_p), ("enter", C.c_void_p),
                ("leave", C.c_void_p)]


def declare(lib):
    RP, SP = C.POINTER(_abi.Request), C.POINTER(_abi.Result)
    GP = C.POINTER(Segment)
    lib.hhmm_segment_workspace_size.argtypes = [RP, C.POINTER(C.c_size_t)]
    lib.hhmm_segment_workspace_size.restype = C.c_int
    lib.hhmm_segment_summary_device.argtypes = [RP, GP, C.c_void_p, C.c_size_t, C.c_void_p]
    lib.hhmm_segment_summary_device.restype = C.c_int
    lib.hhmm_segment_finish_device.argtypes = [RP, SP, GP, C.c_void_p, C.c_size_t, C.c_void_p]
    lib.hhmm_segment_finish_device.restype = C.c_int
    return lib


def slice_time(data, t0, t1):
    """The data block restricted to steps [t0, t1) of every series."""
    out = dict(data)
    for k in ("x", "x_t", "g", "sign"):
        if k in data:
            a = np.atleast_2d(np.asarray(data[k]))
            out[k] = np.asfortranarray(a[:, t0:t1])
    if "T" in out and np.ndim(out["T"]) > 0:
        raise ValueError("segment windows need every series at full length (no data['T'])")
    return out


def windows(T, world):
    """Contiguous [t0, t1) windows of T steps over `world` ranks (lengths differ by <= 1)."""
    q, r = divmod(T, world)
    out, b = [], 0
    for i in range(world):
        e = b + q + (1 if i < r else 0)
        out.append((b, e))
        b = e
    return out


class SegmentWindow:
    """One rank's window [t0, t1) of a batch, resident on `device` (torch).

    The request is built by api.PreparedRequest from the window's numpy
    arrays; every buffer it points at is copied to the device byte for byte
    (the ABI layouts are the arrays' own memory order)."""

    def __init__(self, lib, model, data, draws, pars, first, last, pairing="grid", device=None):
        import torch
        pars = list(pars)
        bad = [p for p in pars if p not in SEGMENT_OUTPUTS]
        if bad:
            raise ValueError(f"{bad}: no segment form (loglik, alpha_tk, beta_tk, ungamma_tk, gamma_tk)")
        self.lib = declare(lib)
        self.dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.pr = api.PreparedRequest(model, data, draws, pars, pairing, flags=_abi.FLAG_SCAN_FORCE)
        self.P, self.K = self.pr.P, self.pr.K
        self.first, self.last = bool(first), bool(last)
        self._dev = []
        host = {a.ctypes.data: a for a in self.pr.keep}
        req = _abi.Request()
        C.memmove(C.byref(req), C.byref(self.pr.req), C.sizeof(req))
        for part in (req.data, req.draws):
            for name, ctype in part._fields_:
                v = getattr(part, name)
                if ctype is C.c_void_p and v is not None:
                    if v not in host:
                        raise RuntimeError(f"request field {name} points at no buffer the request holds")
                    setattr(part, name, self._upload(host[v]))
        self.req = req
        self.res = _abi.Result()
        self.out = {}
        for name in pars:
            arr = self.pr.out[name]
            t = self._upload(arr, keep=False)
            self.out[name] = (arr, t)
            setattr(self.res, name, t.data_ptr())
        self.status = torch.zeros(self.P, dtype=torch.int32, device=self.dev)
        self.res.pair_status = self.status.data_ptr()
        ws = C.c_size_t(0)
        self._check(self.lib.hhmm_segment_workspace_size(C.byref(req), C.byref(ws)))
        self.ws = torch.empty(max(int(ws.value), 256), dtype=torch.uint8, device=self.dev)
        self.nsum = 2 * self.K * self.K + 3

    def _upload(self, arr, keep=True):
        import torch
        flat = np.frombuffer(memoryview(np.ascontiguousarray(arr.ravel(order="K"))).cast("B"), dtype=np.uint8)
        t = torch.from_numpy(flat.copy()).to(self.dev)
        if keep:
            self._dev.append(t)
            return t.data_ptr()
        return t

    def _check(self, st):
        if st < 0:
            raise api.HHMMError(st, self.lib.hhmm_last_error().decode())

    def _stream(self):
        import torch
        return torch.cuda.current_stream(self.dev).cuda_stream

    def summary(self):
        """Launches the summary call; returns the device tensor [2K^2 + 3, P]
        (row f = field f of every pair: SF, SQ, SF exponent, log scale, SQ exponent)."""
        import torch
        s = torch.empty((self.nsum, self.P), dtype=torch.float64, device=self.dev)
        seg = Segment(int(self.first), int(self.last), s.data_ptr(), None, None)
        self._check(self.lib.hhmm_segment_summary_device(C.byref(self.req), C.byref(seg), self.ws.data_ptr(),
                                                         self.ws.numel(), self._stream()))
        return s

    def finish(self, enter=None, leave=None):
        """enter / leave: [K + 1, P] float64 (device or host) for a window that
        is not first / not last.  Returns the window's outputs as host arrays
        shaped like api.gqs before reshaping (P-first, Fortran order), and
        "pair_status" [P]."""
        import torch
        keep = []

        def dev(v):
            if v is None:
                return None
            t = torch.as_tensor(np.asarray(v) if not isinstance(v, torch.Tensor) else v, dtype=torch.float64)
            t = t.to(self.dev).contiguous()
            keep.append(t)
            return t.data_ptr()

        seg = Segment(int(self.first), int(self.last), None, dev(enter), dev(leave))
        self._check(self.lib.hhmm_segment_finish_device(C.byref(self.req), C.byref(self.res), C.byref(seg),
                                                        self.ws.data_ptr(), self.ws.numel(), self._stream()))
        torch.cuda.synchronize(self.dev)
        out = {}
        for name, (arr, t) in self.out.items():
            flat = np.frombuffer(t.cpu().numpy().tobytes(), dtype=arr.dtype)
            out[name] = np.ndarray(arr.shape, dtype=arr.dtype, buffer=flat.copy(),
                                   order="F" if arr.flags.f_contiguous else "C")
        # per pair: HHMM_PAIR_INVALID_DATA where this window's data, or a chained
        # summary of another window (a NaN log scale), breaks a data-block bound
        out["pair_status"] = self.status.cpu().numpy()
        return out


def _renorm(v, sc):
    """v / max(v) per pair (columns), the log of the max added to sc."""
    m = np.max(v, axis=0)
    m = np.where(m > 0, m, 1.0)
    return v / m, sc + np.log(m)


def boundaries(summaries, K):
    """Chains the windows' summaries ([2K^2 + 3, P] each, window order) into
    the state entering every window, beta leaving every window ([K + 1, P]:
    the vector up to scale, then its log scale; None where the window is the
    first / the last) and the log-likelihood of the whole series per pair."""
    R = len(summaries)
    sums = [np.asarray(s, dtype=np.float64) for s in summaries]
    P = sums[0].shape[1]
    KK = K * K

    def SF(r):  # [P, K, K]
        return sums[r][:KK].T.reshape(P, K, K)

    def SQ(r):
        return sums[r][KK:2 * KK].T.reshape(P, K, K)

    enter = [None] * R
    f = SF(0)[:, 0, :].T.copy()  # [K, P]: the first window's rows all hold the state leaving it
    sc = sums[0][2 * KK + 1] + LN2 * sums[0][2 * KK]
    f, sc = _renorm(f, sc)
    for r in range(1, R):
        enter[r] = np.vstack([f, sc[None]])
        f = np.einsum("pi,pij->jp", f.T, SF(r))
        sc = sc + sums[r][2 * KK + 1] + LN2 * sums[r][2 * KK]
        f, sc = _renorm(f, sc)
    loglik = np.log(f.sum(axis=0)) + sc
    leave = [None] * R
    b = np.ones((K, P))
    bsc = np.zeros(P)
    for r in range(R - 1, 0, -1):
        b = np.einsum("pij,jp->ip", SQ(r), b)
        bsc = bsc + sums[r][2 * KK + 1] + LN2 * sums[r][2 * KK + 2]
        b, bsc = _renorm(b, bsc)
        leave[r - 1] = np.vstack([b, bsc[None]])
    return enter, leave, loglik
