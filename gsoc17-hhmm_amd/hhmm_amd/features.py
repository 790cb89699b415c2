"""Host mirror of the reference's feature extractor.

The reference calls
    zig <- extract_features(tdata, features.alpha)    # tayal2009/main.R:61, R/wf-trade.R:58
on an xts of PRICE and SIZE (tayal2009/R/feature-extraction.R:8-133) and codes
the leg feature for the Tayal HHMM as
    sign = ifelse(x < L + 1, 1, 2); x = ifelse(x < L + 1, x, x - L)   # tayal2009/main.R:85-89
`extract_features()` below is that call on the gfx950 engine
(include/hhmm_features.h): it returns the zig-zag table as a dict of columns
(price, start, end, size_av, f0, f1, f2, feature, trend) plus the Tayal data
coding (x, sign).  There is no CPU fallback.
"""
import ctypes as C

import numpy as np

COLUMNS = {"price": "f64", "start": "i32", "end": "i32", "size_av": "f64", "f0": "i32", "f1": "i32",
           "f2": "i32", "feature": "i32", "trend": "i32", "x": "i32", "sign": "i32"}


class Ticks(C.Structure):
    _fields_ = [
        ("n", C.c_int64),
        ("price", C.c_void_p),
        ("size", C.c_void_p),
        ("time", C.c_void_p),
        ("alpha", C.c_double),
    ]


class Legs(C.Structure):
    _fields_ = [("capacity", C.c_int64), ("n_legs", C.c_int64)] + [(k, C.c_void_p) for k in COLUMNS]


def declare(lib):
    lib.hhmm_extract_features.argtypes = [C.POINTER(Ticks), C.POINTER(Legs), C.c_int]
    lib.hhmm_extract_features.restype = C.c_int
    lib.hhmm_features_workspace_size.argtypes = [C.c_int64, C.POINTER(C.c_size_t)]
    lib.hhmm_features_workspace_size.restype = C.c_int
    lib.hhmm_extract_features_device.argtypes = [C.POINTER(Ticks), C.POINTER(Legs), C.c_void_p, C.c_size_t,
                                                 C.c_void_p]
    lib.hhmm_extract_features_device.restype = C.c_int
    return lib


def make_ticks(price, size, time, alpha=0.25):
    """Ticks struct over contiguous float64 copies (returned to keep them alive)."""
    keep = [np.ascontiguousarray(a, dtype=np.float64) for a in (price, size, time)]
    n = keep[0].size
    if keep[1].size != n or keep[2].size != n:
        raise ValueError("price, size and time must have the same length")
    tk = Ticks(n, keep[0].ctypes.data, keep[1].ctypes.data, keep[2].ctypes.data, float(alpha))
    tk._keep = keep
    return tk, keep


def make_legs(capacity):
    out = {k: np.zeros(max(capacity, 1), dtype=np.float64 if t == "f64" else np.int32)
           for k, t in COLUMNS.items()}
    legs = Legs(capacity, 0, *[out[k].ctypes.data for k in COLUMNS])
    return legs, out


def extract_features(price, size, time, alpha=0.25, device=-1, lib=None):
    """extract_features(tdata, alpha) on the GPU -> {column: array[n_legs]}."""
    from .api import HHMMError, load_library
    lib = declare(lib or load_library())
    tk, _keep = make_ticks(price, size, time, alpha)
    legs, out = make_legs(tk.n)
    st = lib.hhmm_extract_features(C.byref(tk), C.byref(legs), int(device))
    if st < 0:
        raise HHMMError(st, lib.hhmm_last_error().decode())
    m = legs.n_legs
    return {k: v[:m].copy() for k, v in out.items()}


def synth_ticks(n, seed=9000, tick=0.01, p0=20.0):
    """Synthetic tick series shaped like the reference's TSX ticks
    (tayal2009/data, CC-BY-NC, not redistributed): a price random walk on a
    one-cent grid with runs of unchanged prices, integer board-lot sizes, and
    increasing POSIXct times with exponential gaps at microsecond resolution
    (gaps up to hours, so difftime's unit switching is exercised)."""
    g = np.random.Generator(np.random.Philox(key=seed))
    steps = g.choice(np.array([-2, -1, 0, 0, 0, 1, 2]), size=n)
    cents = np.round(p0 / tick) + np.cumsum(steps)
    price = cents * tick
    size = 100.0 * g.integers(1, 50, size=n)
    gaps = np.round(g.exponential(3.0, size=n) * 1e6) / 1e6
    gaps[g.random(n) < 0.002] *= 1500.0  # occasional long pauses (mins / hours)
    time = 1178020800.0 + np.cumsum(gaps)  # 2007-05-01 (tayal2009/data file dates)
    return price, size, time


def index_ticks(legs, price):
    """0-based tick of each zig-zag row's xts index.

    The reference builds the table as `price[which(direction.chg) - 1, ]`
    (feature-extraction.R:30), so row n carries the time of the tick before the
    n-th change point: the leg's own end for every row but the last (whose end
    is overwritten with nrow(price), :36).  The last change point is found
    again from the prices (host side, O(n))."""
    end = np.asarray(legs["end"], dtype=np.int64)
    m = end.size
    out = np.empty(m, dtype=np.int64)
    if m == 0:
        return out
    out[:-1] = end[:-1] - 1
    p = np.asarray(price, dtype=np.float64)
    d = np.sign(np.diff(p))                      # direction of ticks 2..n (:20-24)
    prev = np.concatenate([[0.0], d[:-1]])       # lag(direction); tick 1 is direction.lt
    chg = np.flatnonzero((d != 0) & (d != prev)) + 1  # 0-based ticks where direction.chg
    out[-1] = chg[-1] - 1
    return out


def xts_window(times, spec, tz="America/Toronto"):
    """Boolean mask of the rows an xts ISO-8601 range subset `x[spec]` keeps,
    e.g. '2007-05-04 09:30:00/2007-05-10 16:30:00' in the index's time zone
    (tayal2009/main.Rmd:73, :406; indexTZ set at main.R:52): from the first
    instant through the end of the last second named."""
    import datetime
    import zoneinfo
    zone = zoneinfo.ZoneInfo(tz)
    lo_s, hi_s = spec.split("/")

    def epoch(s):
        return datetime.datetime.strptime(s.strip(), "%Y-%m-%d %H:%M:%S").replace(tzinfo=zone).timestamp()

    lo, hi = epoch(lo_s), epoch(hi_s) + 1.0
    t = np.asarray(times, dtype=np.float64)
    return (t >= lo) & (t < hi)
