"""GPU: every committed golden fixture (tests/golden/*.npz) through the HIP
path.  The fixtures hold seeded inputs and the oracle's outputs (made by
tests/golden/make_golden.py after the independent Python transcription
agreed); here the gfx950 engine must reproduce them: paths, statuses and
pair_status bit-exact, floats within tests/tolerances.py.  The HMM-family
fixtures also run through the parallel scan over T (forced 4- and 8-step
chunks) and the exact T-parallel Viterbi (forced), so each schedule meets
the same vectors."""
import numpy as np
import pytest

from hhmm_amd import _abi
from test_golden import MODELS, load
from tolerances import compare

pytestmark = pytest.mark.gpu

HMM_FAMILY = {"hmm", "hmm-multinom", "hmm-multinom-semisup", "hhmm-tayal2009", "hhmm-tayal2009-lite"}
SCHEDULES = {
    "default": 0,
    "scan8": _abi.FLAG_SCAN_FORCE | _abi.flag_scan_chunk_log2(3),
    "scan4": _abi.FLAG_SCAN_FORCE | _abi.flag_scan_chunk_log2(2),
    "vscan": _abi.FLAG_VIT_SCAN,
    "vit-lanes": _abi.FLAG_VIT_LANES,
    "vit-states": _abi.FLAG_VIT_STATES,
    "vfb": _abi.FLAG_VIT_LANES | _abi.FLAG_VFB,
}


def _cases():
    for m in MODELS:
        for name in SCHEDULES:
            if name != "default" and m not in HMM_FAMILY:
                continue
            yield m, name


@pytest.mark.parametrize("model,schedule", list(_cases()), ids=[f"{m}-{s}" for m, s in _cases()])
def test_engine_reproduces_golden(engine, model, schedule):
    import hhmm_amd
    data, draws, outs = load(model)
    flags = SCHEDULES[schedule]
    pars = [k for k in outs if k != "pair_status"]
    if schedule.startswith("scan"):
        # the T-scan evaluates the probability-space profile (log-scale outputs stay sequential)
        pars = [k for k in pars if k not in ("unalpha_tk", "unbeta_tk", "unalpha_tk_oos")]
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, return_status=True, flags=flags)
    for k in pars + ["pair_status"]:
        compare(k, got[k], outs[k])
