"""Walk-forward batch assembly: the reference's 204 separate
Stan fits as ONE batched request.

The reference walks a window forward over every stock's trading days
(tayal2009/test-strategy.R:45-59): each task is `window_ins + window_oos`
consecutive day files, an in-sample span and an out-of-sample span.
wf_trade() then, per task and in its own R worker (tayal2009/R/wf-trade.R:
30-100): loads and rbinds the files, `na.omit`s PRICE/SIZE, runs
extract_features(tdata, alpha), keeps the in-sample legs `zig[ins]` and every
leg after the last of them as out-of-sample, codes the 18-symbol feature as
(x, sign) and fits hhmm-tayal2009-lite.stan with its own posterior draws.

Here the per-task steps map onto the engine:
  window_tasks()  the task list of test-strategy.R (files, ins / oos spans);
  window_data()   wf-trade.R:53-87 for one task: features -> stan.data;
  assemble()      every window as one series of a ragged request, each with
                  its own block of draws (HHMM_PAIR_BLOCK: pair p = b + B*n
                  evaluates window n under draw p), so one hhmm_run evaluates
                  all fits' generated quantities at once;
  split()         the batched outputs back into per-window extract()-shaped
                  arrays ([B, T_n, K] / [B, T_n] / [B]).
"""
import pathlib

import numpy as np

from . import features as F
from . import rdata

L_TAYAL = 9  # tayal2009/test-strategy.R:9


def _day(name):
    """'2007.05.01.G.TO.RData' -> '2007-05-01' (filename_to_timestamp, test-strategy.R:37-44)."""
    return name[:10].replace(".", "-")


def window_tasks(data_path, window_ins=5, window_oos=1):
    """test-strategy.R:45-59: for every stock directory `*.TO` under data_path
    and every run of window_ins + window_oos consecutive day files, the task
    (files, ins span, oos span) with spans '<day> 09:30:00/<day> 16:30:00'."""
    root = pathlib.Path(data_path)
    out = []
    for d in sorted(p for p in root.iterdir() if p.is_dir() and p.name.endswith(".TO")):
        files = sorted(f.name for f in d.iterdir())
        w = window_ins + window_oos
        for i in range(len(files) - w + 1):
            out.append({
                "stock": d.name,
                "files": [d / f for f in files[i:i + w]],
                "ins": f"{_day(files[i])} 09:30:00/{_day(files[i + window_ins - 1])} 16:30:00",
                "oos": f"{_day(files[i + window_ins])} 09:30:00/{_day(files[i + w - 1])} 16:30:00",
            })
    return out


def window_data(price, size, time, ins, alpha=0.25, extract=None, L=L_TAYAL):
    """wf-trade.R:53-87 for one task's ticks: extract_features, the in-sample
    legs zig[ins] (index in America/Toronto), every later leg as out-of-sample
    (`zig[(last(ind) + 1):nrow(zig)]`, :60), and the Tayal coding
    sign = x <= L ? 1 : 2, x = x <= L ? x : x - L (:79-86).
    `extract` defaults to the gfx950 extractor (hhmm_amd.features)."""
    legs = (extract or F.extract_features)(price, size, time, alpha)
    when = np.asarray(time)[F.index_ticks(legs, price)]
    ind = np.flatnonzero(F.xts_window(when, ins))
    if ind.size == 0:
        raise ValueError(f"no zig-zag leg inside {ins}")
    feat = np.asarray(legs["feature"], dtype=np.int32)
    fi, fo = feat[ind], feat[ind[-1] + 1:]

    def code(f):
        return np.where(f <= L, f, f - L).astype(np.int32), np.where(f <= L, 1, 2).astype(np.int32)

    x, sign = code(fi)
    x_oos, sign_oos = code(fo)
    return {"x": x, "sign": sign, "x_oos": x_oos, "sign_oos": sign_oos}


def load_window(task, alpha=0.25, extract=None):
    """One task from its RData files (rbind + na.omit, wf-trade.R:41-51)."""
    price, size, time = rdata.load_ticks(task["files"])
    return window_data(price, size, time, task["ins"], alpha, extract)


def assemble(windows, draws, K=4, L=L_TAYAL):
    """(data, draws) of ONE hhmm-tayal2009-lite request over every window.

    windows: list of stan.data dicts (x, sign, x_oos, sign_oos), ragged.
    draws:   list of per-window draw dicts (p_11 [B], A_row [B, 2, 2],
             phi_k [B, K, L]) with the same B for every window.
    Series n is window n (T, T_oos ragged, padded with a valid symbol);
    the draws are concatenated window-major: draw b of window n is p = b + B*n,
    the layout HHMM_PAIR_BLOCK pairs with series n."""
    N = len(windows)
    if N == 0 or len(draws) != N:
        raise ValueError("one draw block per window")
    B = np.asarray(draws[0]["p_11"]).shape[0]
    T = np.array([w["x"].size for w in windows], dtype=np.int32)
    To = np.array([w["x_oos"].size for w in windows], dtype=np.int32)
    if (T < 1).any() or (To < 1).any():
        raise ValueError("every window needs T >= 1 and T_oos >= 1 (int<lower=1> T, T_oos)")
    x = np.ones((N, T.max()), dtype=np.int32)
    sg = np.ones((N, T.max()), dtype=np.int32)
    xo = np.ones((N, To.max()), dtype=np.int32)
    so = np.ones((N, To.max()), dtype=np.int32)
    for n, w in enumerate(windows):
        x[n, :T[n]], sg[n, :T[n]] = w["x"], w["sign"]
        xo[n, :To[n]], so[n, :To[n]] = w["x_oos"], w["sign_oos"]
    data = {"K": K, "L": L, "x": x, "sign": sg, "T": T, "x_oos": xo, "sign_oos": so, "T_oos": To}
    out = {}
    for k in draws[0]:
        blocks = [np.asarray(d[k], dtype=np.float64) for d in draws]
        if any(b.shape[0] != B for b in blocks):
            raise ValueError(f"draw array {k}: every window needs the same number of draws ({B})")
        out[k] = np.concatenate(blocks, axis=0)
    return data, out


def split(result, data):
    """Batched outputs (pair-major, ABI order) -> one dict per window with the
    extract() shapes of that window's own fit: [B, T_n, ...] over its T_n
    (in-sample) or T_oos_n (out-of-sample) steps."""
    T, To = np.asarray(data["T"]), np.asarray(data["T_oos"])
    N = T.size
    P = next(np.asarray(v).shape[0] for k, v in result.items() if k not in ("status",))
    B = P // N
    per = []
    for n in range(N):
        sl = slice(n * B, (n + 1) * B)
        d = {}
        for k, v in result.items():
            if k == "status":
                continue
            v = np.asarray(v)
            if v.ndim == 1:
                d[k] = v[sl]
            else:
                steps = To[n] if k.endswith("_oos") or (k in ("zstar_t",)) else T[n]
                d[k] = v[sl, :steps]
        per.append(d)
    return per
