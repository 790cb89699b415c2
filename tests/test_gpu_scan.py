"""GPU: the parallel scan over T against the CPU oracle.

The scan (chunk transfer products -> boundary scan -> per-chunk sweeps) is
forced with small T-chunks so that short, oracle-sized series cross many
chunk boundaries; results must agree with the sequential reference within
the tolerances of tests/tolerances.py, and the Viterbi path (sequential in
either case) stays bit-exact.  At full size the scan is checked against the
engine's own sequential path (a size-independent property: the same
posteriors whichever way T is split).
"""
import numpy as np
import pytest

from hhmm_amd import _abi, synth
from tolerances import compare_all

pytestmark = pytest.mark.gpu

SCAN_MODELS = ["hmm", "hmm-multinom", "hmm-multinom-semisup", "hhmm-tayal2009"]


def force(log2):
    return _abi.FLAG_SCAN_FORCE | _abi.flag_scan_chunk_log2(log2)


@pytest.mark.parametrize("model", SCAN_MODELS)
@pytest.mark.parametrize("T,log2", [(1, 4), (2, 4), (37, 4), (130, 5), (1000, 6), (1000, 3)])
def test_scan_matches_oracle(engine, oracle, model, T, log2):
    import hhmm_amd
    data, draws = synth.GENERATORS[model](N=2, S=40, T=T)
    pars = synth.PARS[model]
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, flags=force(log2), return_status=True)
    ref = oracle.gqs(model, data, draws, pars=pars, return_status=True)
    compare_all(got, ref, pars + ["pair_status"])


@pytest.mark.parametrize("model,kw", [("hmm", dict(K=6)), ("hmm-multinom", dict(K=8, L=9)),
                                      ("hmm-multinom", dict(K=1, L=3)), ("hmm-multinom-semisup", dict(K=4))])
def test_scan_other_K(engine, oracle, model, kw):
    import hhmm_amd
    data, draws = synth.GENERATORS[model](N=2, S=33, T=301, **kw)
    pars = ["loglik", "gamma_tk", "unalpha_tk", "unbeta_tk", "alpha_tk", "beta_tk"]
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, flags=force(4))
    ref = oracle.gqs(model, data, draws, pars=pars)
    compare_all(got, ref, pars)


@pytest.mark.parametrize("model", SCAN_MODELS)
def test_scan_ragged(engine, oracle, model):
    import hhmm_amd
    N, S, T = 5, 24, 700
    data, draws = synth.GENERATORS[model](N=N, S=S, T=T)
    data["T"] = np.array([700, 1, 65, 64, 333], dtype=np.int32)
    pars = ["loglik", "gamma_tk", "alpha_tk", "zstar_t"]
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, flags=force(6))
    ref = oracle.gqs(model, data, draws, pars=pars)
    compare_all(got, ref, pars)


def test_scan_auto_long_series_matches_sequential(engine):
    """C5-shaped batches (few pairs, long T): the automatic scan and the forced
    sequential path of the engine agree (posteriors, loglik; the path is the
    same sequential Viterbi)."""
    import hhmm_amd
    data, draws = synth.hmm_multinom(N=2, S=64, T=200_000)
    pars = ["loglik", "gamma_tk", "zstar_t"]
    scan = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine)
    seq = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine, flags=_abi.FLAG_SCAN_OFF)
    compare_all(scan, seq, pars)


def test_scan_auto_long_tayal_matches_sequential(engine):
    """Tayal on a long series: the reference's forward and backward masks
    disagree, so alpha and beta drift onto different
    states and gamma = normalize(alpha .* beta) becomes 0/0 = NaN once their
    overlap underflows (the oracle shows it from t ~ 2000 on these inputs).
    Both engine paths reproduce it; placements may differ only where the
    overlap sits at the underflow threshold.  Everywhere else they agree."""
    import hhmm_amd
    data, draws = synth.tayal(N=2, S=64, T=200_000)
    pars = ["loglik", "gamma_tk", "zstar_t"]
    scan = hhmm_amd.gqs("hhmm-tayal2009", data, draws, pars=pars, lib=engine)
    seq = hhmm_amd.gqs("hhmm-tayal2009", data, draws, pars=pars, lib=engine, flags=_abi.FLAG_SCAN_OFF)
    compare_all(scan, seq, ["loglik", "zstar_t"])
    g1, g2 = scan["gamma_tk"], seq["gamma_tk"]
    n1, n2 = np.isnan(g1).any(axis=2), np.isnan(g2).any(axis=2)
    assert (n1 != n2).mean() < 1e-5
    ok = ~(n1 | n2)
    from tolerances import compare
    compare("gamma_tk", g1[ok], g2[ok])


@pytest.mark.parametrize("model", SCAN_MODELS)
@pytest.mark.parametrize("S", [250, 65, 1])
def test_scan_pairs_not_whole_waves(engine, oracle, model, S):
    """Pair counts that are not a multiple of the 64-lane wave: the per-chunk
    sweep pads each T-chunk's lanes to whole waves, so no wave spans two
    chunks (a wave that did once read checkpoint rows past its chunk's)."""
    import hhmm_amd
    data, draws = synth.GENERATORS[model](N=1, S=S, T=600)
    pars = ["loglik", "gamma_tk", "zstar_t", "logp_zstar"]
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, flags=force(4))
    ref = oracle.gqs(model, data, draws, pars=pars)
    compare_all(got, ref, pars)


def test_scan_c5_shape_many_chunks(engine):
    """C5's lane shape (250 pairs) across hundreds of T-chunks: the scan agrees
    with the sequential sweep."""
    import hhmm_amd
    data, draws = synth.hmm_multinom(N=1, S=250, T=30_000)
    pars = ["loglik", "gamma_tk"]
    scan = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine, flags=force(6))
    seq = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine, flags=_abi.FLAG_SCAN_OFF)
    compare_all(scan, seq, pars)
