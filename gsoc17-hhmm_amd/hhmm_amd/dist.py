"""Multi-GPU sharding of a batch of (series x draw) pairs.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI).
Pairs are independent -- the reference itself runs one fit per series and
parallelises fits over worker processes (tayal2009/R/wf-trade.R:30-34) -- so
each rank evaluates a contiguous block of SERIES under all S draws, with no
collective on the data path.  The only exchanges are the ones the north star
names: an all-reduce of the per-draw summed log-likelihood and a gather of
the decoded Viterbi paths to rank 0.

`compute` defaults to hhmm_amd.gqs (the gfx950 engine); tests inject the CPU
oracle to exercise the same orchestration under the gloo backend.
"""
import numpy as np


def shard_range(n, world, rank):
    """Contiguous [begin, end) block of n items for `rank` (sizes differ by <= 1)."""
    q, r = divmod(n, world)
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


_SERIES_KEYS = ("x", "x_t", "g", "sign", "u_tm", "T", "x_oos", "sign_oos", "T_oos")


def slice_series(data, b, e):
    """The data block restricted to series [b, e) (series is the first axis)."""
    out = {}
    for k, v in data.items():
        if k in _SERIES_KEYS:
            a = np.asarray(v)
            if k in ("T", "T_oos"):
                out[k] = a.reshape(-1)[b:e]
            elif a.ndim >= 2 or k in ("x", "x_t", "g", "sign", "x_oos", "sign_oos"):
                a = np.atleast_2d(a) if k != "u_tm" else (a if a.ndim == 3 else a[None])
                out[k] = a[b:e]
            else:
                out[k] = a
        else:
            out[k] = v
    return out


def default_device(group=None):
    """Where the collective buffers live: the rank's current GPU under nccl
    (RCCL rejects host tensors), the host under gloo."""
    import torch
    import torch.distributed as dist

    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def slice_draws(draws, b, e):
    return {k: np.asarray(v)[b:e] for k, v in draws.items()}


def pair_range(N, S, pairing, b, e):
    """Global ABI pair range [begin, end) of series block [b, e): contiguous in
    every pairing (grid p = s + S*n, zip p = n, block p = j + B*n)."""
    per = {"grid": S, "zip": 1, "block": S // N if N else 0}[pairing]
    return b * per, e * per


def gqs_sharded(model, data, draws, pars, pairing="grid", compute=None, group=None, device=None,
                paths_out=None):
    """Evaluates this rank's shard and performs the two exchanges.

    Returns (local, summed_loglik, paths):
      local          this rank's outputs (pairs of its series block, ABI order)
      summed_loglik  [S] per-draw log-likelihood summed over ALL series (all-reduce
                     of a device tensor under nccl; zip / block pairing: each
                     draw's own series)
      paths          zstar_t of every pair in global ABI order:
                     * paths_out given (an array of shape (P, T) that every rank
                       can write, e.g. a np.memmap on the node's shared memory):
                       each rank writes its own contiguous pair slice into it
                       (SURVEY §8e's direct per-rank copy into the caller's
                       buffer; no collective moves the paths); returns paths_out
                       on every rank after a barrier;
                     * otherwise a tensor gather to rank 0 (padded device tensors
                       under nccl, no pickling); rank 0 gets the array, others None.
    """
    import torch
    import torch.distributed as dist

    if compute is None:
        from .api import gqs as compute
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    xkey = "x_t" if model.startswith("iohmm") else "x"
    N = np.atleast_2d(np.asarray(data[xkey])).shape[0] if np.asarray(data[xkey]).ndim > 1 or \
        not model.startswith("iohmm") else 1
    S = next(np.asarray(v).shape[0] for v in draws.values())
    if pairing == "block" and S % N:
        raise ValueError(f"block pairing needs n_draws ({S}) to be a multiple of n_series ({N})")
    if pairing == "zip" and S != N:
        raise ValueError(f"zip pairing needs n_draws ({S}) == n_series ({N})")
    b, e = shard_range(N, world, rank)
    ldata = slice_series(data, b, e)
    B = S // N if pairing == "block" else 1  # draws per series (block pairing: one fit per series)
    ldraws = draws if pairing == "grid" else slice_draws(draws, b * B, e * B)
    local = compute(model, ldata, ldraws, pars=pars, pairing=pairing) if e > b else {}

    dev = device if device is not None else default_device(group)
    summed = None
    if "loglik" in pars:
        s_len = S if pairing in ("grid", "block") else N
        acc = torch.zeros(s_len, dtype=torch.float64, device=dev)
        if e > b:
            ll = np.asarray(local["loglik"])
            if pairing == "grid":  # pair p = s + S*n -> (S, n_local)
                acc += torch.from_numpy(ll.reshape((S, e - b), order="F").sum(axis=1)).to(dev)
            else:  # zip: pair = series = draw; block: pair = draw, this rank's draws [b*B, e*B)
                acc[b * B:e * B] += torch.from_numpy(ll).to(dev)
        dist.all_reduce(acc, group=group)
        summed = acc.cpu().numpy()

    paths = None
    if "zstar_t" in pars:
        p0, p1 = pair_range(N, S, pairing, b, e)
        if paths_out is not None:
            if e > b:
                paths_out[p0:p1] = np.asarray(local["zstar_t"])
            dist.barrier(group=group)
            return local, summed, paths_out
        T = int(np.asarray(local["zstar_t"]).shape[1]) if e > b else 0
        T = int(_all_max(T, dev, group))
        rows = [pair_range(N, S, pairing, *shard_range(N, world, r)) for r in range(world)]
        cap = max(r1 - r0 for r0, r1 in rows)
        buf = torch.zeros((cap, T), dtype=torch.int32, device=dev)
        if e > b:
            buf[:p1 - p0] = torch.from_numpy(np.ascontiguousarray(local["zstar_t"])).to(dev)
        bufs = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
        dist.gather(buf, bufs, dst=0, group=group)
        if rank == 0:
            paths = np.concatenate([g[:r1 - r0].cpu().numpy() for g, (r0, r1) in zip(bufs, rows)], axis=0)
            paths = np.asfortranarray(paths)
    return local, summed, paths


def _all_max(v, dev, group):
    import torch
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def gqs_tsplit(model, data, draws, pars, group=None, pairing="grid", lib=None):
    """One batch whose series are split along T over the ranks (SURVEY.md §8e:
    a single very long series -- C5's shape when pairs are few).  Rank r holds
    the steps [t0, t1) of every series (segment.windows); it computes its
    window's K x K summaries on its GPU (hhmm_segment_summary_device),
    all-gathers them (2K^2 + 3 doubles per pair and rank -- RCCL over xGMI
    under nccl), chains them into the state entering and beta leaving its
    window, and finishes its window (phases 2-3 of the T-scan).

    Returns (window, outputs, loglik): window = (t0, t1); outputs = the
    window's requested [P, t1 - t0, ...] arrays (P-first, as api.PreparedRequest
    lays them out) and "pair_status" [P] (HHMM_PAIR_INVALID_DATA where any
    rank's window breaks a data-block bound: its summary carries a NaN log
    scale, and loglik is NaN for that pair); loglik = the whole series' log-likelihood per pair (every
    rank computes it from the same gathered summaries)."""
    import torch
    import torch.distributed as dist

    from . import api, segment

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    x = np.atleast_2d(np.asarray(data["x_t" if "x_t" in data else "x"]))
    if x.shape[-1] < world:  # every rank holds the same data, so every rank raises here
        raise ValueError(f"gqs_tsplit: T = {x.shape[-1]} is shorter than the world size {world}")
    wins = segment.windows(x.shape[-1], world)
    t0, t1 = wins[rank]
    dev = default_device(group)
    # a rank whose window fails must not leave the others waiting in all_gather:
    # agree on success first
    err, s, win = None, None, None
    try:
        lib = lib or api.load_library()
        win = segment.SegmentWindow(lib, model, segment.slice_time(data, t0, t1), draws,
                                    list(dict.fromkeys(["loglik"] + list(pars))), rank == 0, rank == world - 1,
                                    pairing)
        s = win.summary()
        torch.cuda.synchronize(win.dev)
    except Exception as ex:  # re-raised below, after every rank knows
        err = ex
    failed = torch.tensor([0 if err is None else 1], dtype=torch.int64, device=dev)
    dist.all_reduce(failed, op=dist.ReduceOp.MAX, group=group)
    if err is not None:
        raise err
    if int(failed.item()):
        raise RuntimeError("gqs_tsplit: the window of another rank failed")
    s = s.to(dev)
    gathered = [torch.empty_like(s) for _ in range(world)]
    dist.all_gather(gathered, s, group=group)
    enter, leave, loglik = segment.boundaries([g.cpu().numpy() for g in gathered], win.K)
    out = win.finish(enter[rank], leave[rank])
    return (t0, t1), out, loglik
