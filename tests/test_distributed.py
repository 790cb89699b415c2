"""World size 2 over gloo: the multi-GPU orchestration (hhmm_amd.dist).

Each rank evaluates its block of series under every draw (no data-path
collective); the per-draw summed log-likelihood is all-reduced and the
Viterbi paths either gathered to rank 0 as tensors or written by every rank
into its slice of a shared caller buffer (np.memmap).  The compute function
is the CPU oracle in the CPU tests and the gfx950 engine (hhmm_amd.gqs) in
the `gpu` test; bench.py uses the same weak-scaling decomposition over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _sizes(pairing, n=5):
    return n, {"zip": n, "grid": 4, "block": 3 * n}[pairing]


def _worker(rank, world, port, model, pairing, q, engine, mmap_path):
    import sys
    import pathlib
    repo = pathlib.Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(repo / "gsoc17-hhmm_amd"), str(repo / "oracle")]
    import torch.distributed as dist
    from hhmm_amd import dist as hdist, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, S = _sizes(pairing)
        data, draws = synth.GENERATORS[model](N=n, S=S, T=30)
        pars = ["loglik", "gamma_tk", "zstar_t"] if model != "hhmm-tayal2009-lite" else ["loglik", "zstar_t"]
        if engine:
            import torch  # noqa: F401  (its HIP runtime first, as in hhmm_amd.api)
            import hhmm_amd
            lib = hhmm_amd.load_library()

            def compute(m, d, w, pars, pairing):
                return hhmm_amd.gqs(m, d, w, pars=pars, pairing=pairing, lib=lib)
        else:
            import pyoracle

            def compute(m, d, w, pars, pairing):
                return pyoracle.gqs(m, d, w, pars=pars, pairing=pairing)

        out = None
        if mmap_path:
            P = {"grid": n * S, "zip": n, "block": S}[pairing]
            out = np.lib.format.open_memmap(mmap_path, mode="r+", dtype=np.int32, shape=(P, 30))
        local, summed, paths = hdist.gqs_sharded(model, data, draws, pars, pairing=pairing, compute=compute,
                                                 paths_out=out)
        q.put((rank, summed, None if mmap_path else paths))
    finally:
        dist.destroy_process_group()


def _run(oracle, model, pairing, engine=False, mmap_path=None):
    from hhmm_amd import synth
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, model, pairing, q, engine, mmap_path))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, summed, paths = q.get(timeout=180)
        res[r] = (summed, paths)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n, S = _sizes(pairing)
    data, draws = synth.GENERATORS[model](N=n, S=S, T=30)
    ref = oracle.gqs(model, data, draws, pars=["loglik", "zstar_t"], pairing=pairing)
    want = ref["loglik"].reshape((S, n), order="F").sum(axis=1) if pairing == "grid" else ref["loglik"]
    for r in range(world):
        np.testing.assert_allclose(res[r][0], want, rtol=1e-13)
    if mmap_path:
        assert np.array_equal(np.load(mmap_path), ref["zstar_t"])
    else:
        assert res[1][1] is None
        assert np.array_equal(res[0][1], ref["zstar_t"])


@pytest.mark.parametrize("model,pairing", [("hmm-multinom", "grid"), ("hmm-multinom", "zip"),
                                           ("hmm-multinom", "block"), ("hhmm-tayal2009-lite", "grid"),
                                           ("iohmm-hmix", "grid")])
def test_two_rank_sharding_matches_single_process(oracle, model, pairing):
    _run(oracle, model, pairing)


@pytest.mark.parametrize("pairing", ["grid", "block"])
def test_two_rank_paths_into_shared_caller_buffer(oracle, tmp_path, pairing):
    """Every rank writes its contiguous pair slice straight into the caller's
    (P, T) array -- a memmap both processes open -- with no collective."""
    n, S = _sizes(pairing)
    P = {"grid": n * S, "zip": n, "block": S}[pairing]
    path = str(tmp_path / "paths.npy")
    np.lib.format.open_memmap(path, mode="w+", dtype=np.int32, shape=(P, 30))[:] = -1
    _run(oracle, "hmm-multinom", pairing, mmap_path=path)


@pytest.mark.gpu
@pytest.mark.parametrize("pairing", ["grid", "block"])
def test_two_rank_sharding_with_the_engine(oracle, pairing):
    """The same orchestration with the gfx950 engine as `compute` (two ranks
    on the box's one GPU, gloo for the exchanges)."""
    _run(oracle, "hmm-multinom", pairing, engine=True)


def test_block_pairing_rejects_ragged_draws():
    from hhmm_amd import dist as hdist, synth
    import torch.distributed as dist
    data, draws = synth.hmm_multinom(N=3, S=7, T=5)
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ["MASTER_PORT"] = str(_free_port())
        dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        with pytest.raises(ValueError, match="multiple"):
            hdist.gqs_sharded("hmm-multinom", data, draws, ["loglik"], pairing="block", compute=lambda *a, **k: {})
    finally:
        dist.destroy_process_group()


def test_shard_range_covers_everything():
    from hhmm_amd.dist import shard_range
    for n in (0, 1, 7, 8, 1000, 1_000_003):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _tsplit_worker(rank, world, port, T, q):
    import sys
    import pathlib
    repo = pathlib.Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(repo / "gsoc17-hhmm_amd"), str(repo / "oracle")]
    import torch.distributed as dist
    from hhmm_amd import dist as hdist, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        try:
            data, draws = synth.GENERATORS["hmm"](N=1, S=3, T=T)
            hdist.gqs_tsplit("hmm", data, draws, ["loglik", "gamma_tk"])
            q.put((rank, "ok"))
        except Exception as ex:  # noqa: BLE001 -- the test inspects what each rank raised
            q.put((rank, type(ex).__name__))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("T", [1, 40])
def test_gqs_tsplit_fails_on_every_rank_without_hanging(T):
    """a rank whose window fails (T shorter than the world; here on
    the CPU box also no gfx950 device) must not leave the other rank waiting in
    all_gather.  Both ranks raise, and the test ends within the queue timeout."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tsplit_worker, args=(r, world, port, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    if T == 1:
        assert got == {0: "ValueError", 1: "ValueError"}
    else:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present: the windows succeed")
        assert "ok" not in got.values() and set(got) == {0, 1}
