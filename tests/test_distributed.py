"""CPU, world_size 2 over gloo: the multi-GPU orchestration (hhmm_amd.dist).

Each rank evaluates its block of series under every draw (no data-path
collective); the per-draw summed log-likelihood is all-reduced and the
Viterbi paths are gathered to rank 0.  The compute function is the CPU
oracle here; on the GPU box it is the gfx950 engine (bench.py uses the same
weak-scaling decomposition over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, model, pairing, q):
    import sys
    import pathlib
    repo = pathlib.Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(repo / "gsoc17-hhmm_amd"), str(repo / "oracle")]
    import torch.distributed as dist
    import pyoracle
    from hhmm_amd import dist as hdist, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 5
        data, draws = synth.GENERATORS[model](N=n, S={"zip": n, "grid": 4, "block": 3 * n}[pairing], T=30)
        pars = ["loglik", "gamma_tk", "zstar_t"] if model != "hhmm-tayal2009-lite" else ["loglik", "zstar_t"]

        def compute(m, d, w, pars, pairing):
            return pyoracle.gqs(m, d, w, pars=pars, pairing=pairing)

        local, summed, paths = hdist.gqs_sharded(model, data, draws, pars, pairing=pairing, compute=compute)
        q.put((rank, summed, paths))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model,pairing", [("hmm-multinom", "grid"), ("hmm-multinom", "zip"),
                                           ("hmm-multinom", "block"), ("hhmm-tayal2009-lite", "grid"),
                                           ("iohmm-hmix", "grid")])
def test_two_rank_sharding_matches_single_process(oracle, model, pairing):
    from hhmm_amd import synth
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, model, pairing, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, summed, paths = q.get(timeout=120)
        res[r] = (summed, paths)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 5
    data, draws = synth.GENERATORS[model](N=n, S={"zip": n, "grid": 4, "block": 3 * n}[pairing], T=30)
    ref = oracle.gqs(model, data, draws, pars=["loglik", "zstar_t"], pairing=pairing)
    S = {"zip": n, "grid": 4, "block": 3 * n}[pairing]
    if pairing == "grid":
        want = ref["loglik"].reshape((S, n), order="F").sum(axis=1)
    else:
        want = ref["loglik"]
    for r in range(world):
        np.testing.assert_allclose(res[r][0], want, rtol=1e-13)
    assert res[1][1] is None
    assert np.array_equal(res[0][1], ref["zstar_t"])


def test_shard_range_covers_everything():
    from hhmm_amd.dist import shard_range
    for n in (0, 1, 7, 8, 1000, 1_000_003):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1
