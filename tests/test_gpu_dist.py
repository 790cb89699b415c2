"""GPU: the multi-GPU orchestration (hhmm_amd.dist) over RCCL with the engine
as `compute`, at world size 1 on the box's one GPU (the driver's 8-GPU node
runs the N > 1 bench; N = 2 is covered over gloo on CPU in
tests/test_distributed.py).  The collective buffers live on the GPU under
nccl; the results equal the single-request engine and the oracle."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("model,pairing", [("hmm-multinom", "grid"), ("hmm-multinom", "zip"),
                                           ("iohmm-hmix", "grid")])
def test_sharded_engine_over_rccl(engine, oracle, model, pairing):
    import torch
    import torch.distributed as dist
    from hhmm_amd import dist as hdist, synth
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        assert hdist.default_device().type == "cuda"
        n = 6
        S = n if pairing == "zip" else 5
        data, draws = synth.GENERATORS[model](N=n, S=S, T=200)
        pars = ["loglik", "gamma_tk", "zstar_t"]
        local, summed, paths = hdist.gqs_sharded(model, data, draws, pars, pairing=pairing)
    finally:
        dist.destroy_process_group()
    ref = oracle.gqs(model, data, draws, pars=pars, pairing=pairing)
    want = ref["loglik"].reshape((S, n), order="F").sum(axis=1) if pairing == "grid" else ref["loglik"]
    np.testing.assert_allclose(summed, want, rtol=1e-12)
    assert np.array_equal(paths, ref["zstar_t"])
    from tolerances import compare
    compare("gamma_tk", local["gamma_tk"], ref["gamma_tk"])
