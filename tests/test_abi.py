"""CPU: the C-ABI shared library (libhhmm.so) loads, exports every entry point
include/hhmm.h declares, and its structs have the layout the header gives
(checked against gcc's offsetof, not just against our own ctypes mirror).
No compute call needs a GPU here; without one the engine must fail loudly."""
import ctypes as C
import pathlib
import re
import subprocess

import numpy as np
import pytest

from hhmm_amd import _abi, api, synth

REPO = pathlib.Path(__file__).resolve().parent.parent
HEADER = REPO / "include" / "hhmm.h"
HEADERS = sorted((REPO / "include").glob("*.h"))


def declared_functions():
    """Every function any include/*.h declares (hhmm.h, hhmm_features.h)."""
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names |= set(re.findall(r"\b(hhmm_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_header_declares_entry_points():
    names = declared_functions()
    for n in ("hhmm_run", "hhmm_run_device", "hhmm_workspace_size", "hhmm_validate", "hhmm_version",
              "hhmm_last_error", "hhmm_init", "hhmm_shutdown", "hhmm_num_pairs", "hhmm_selftest_cr_log",
              "hhmm_selftest_cr_exp", "hhmm_selftest_det_log", "hhmm_selftest_det_exp", "hhmm_extract_features", "hhmm_extract_features_device",
              "hhmm_features_workspace_size", "hhmm_neighbouring_forecast",
              "hhmm_neighbouring_forecast_device", "hhmm_num_unconstrained", "hhmm_constrain_draws",
              "hhmm_constrain_draws_device"):
        assert n in names


def test_library_exports_every_declared_symbol(engine):
    out = subprocess.run(["nm", "-D", "--defined-only", str(api.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (hhmm_\w+)", out))
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    for n in declared_functions():
        getattr(engine, n)  # resolvable through ctypes


def _c_layout(tmp_path):
    from hhmm_amd import features as F
    from hhmm_amd import forecast as Fc
    from hhmm_amd import params as Pm
    fields = {
        "hhmm_ticks": [f[0] for f in F.Ticks._fields_],
        "hhmm_legs": [f[0] for f in F.Legs._fields_],
        "hhmm_forecast_request": [f[0] for f in Fc.ForecastRequest._fields_],
        "hhmm_param_out": [f[0] for f in Pm.ParamOut._fields_],
        "hhmm_data": [f[0] for f in _abi.Data._fields_],
        "hhmm_draws": [f[0] for f in _abi.Draws._fields_],
        "hhmm_request": [f[0] for f in _abi.Request._fields_],
        "hhmm_result": [f[0] for f in _abi.Result._fields_],
    }
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "hhmm.h"', '#include "hhmm_features.h"',
           '#include "hhmm_forecast.h"', '#include "hhmm_params.h"',
           "int main(void){"]
    for st, fs in fields.items():
        src.append(f'printf("{st} sizeof %zu\\n", sizeof({st}));')
        for f in fs:
            src.append(f'printf("{st} {f} %zu\\n", offsetof({st}, {f}));')
    src.append("return 0;}")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(REPO / "include"), str(c), "-o", str(exe)], check=True)
    rows = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    return {tuple(r.split()[:2]): int(r.split()[2]) for r in rows if r}


def test_struct_layout_matches_header(tmp_path):
    lay = _c_layout(tmp_path)
    from hhmm_amd import features as F
    from hhmm_amd import forecast as Fc
    from hhmm_amd import params as Pm
    for cname, cls in (("hhmm_data", _abi.Data), ("hhmm_draws", _abi.Draws), ("hhmm_request", _abi.Request),
                       ("hhmm_result", _abi.Result), ("hhmm_ticks", F.Ticks), ("hhmm_legs", F.Legs),
                       ("hhmm_forecast_request", Fc.ForecastRequest), ("hhmm_param_out", Pm.ParamOut)):
        assert lay[(cname, "sizeof")] == C.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert lay[(cname, f)] == getattr(cls, f).offset, (cname, f)


def _prepared(model="hmm-multinom", **kw):
    data, draws = synth.GENERATORS[model](N=2, S=3, T=10, **kw)
    return api.PreparedRequest(model, data, draws, synth.PARS[model])


def _validate(engine, pr, host=1):
    return engine.hhmm_validate(C.byref(pr.req), C.byref(pr.res), host)


def test_validate_accepts_good_requests(engine):
    for m in synth.GENERATORS:
        pr = _prepared(m)
        assert _validate(engine, pr) == _abi.OK, (m, engine.hhmm_last_error())


def test_validate_rejects_out_of_range_data(engine):
    pr = _prepared()
    pr.keep[0][0, 3] = 10  # x outside 1..L (int<lower=1, upper=L> x[T])
    assert _validate(engine, pr) == _abi.ERR_INVALID_ARGUMENT
    assert b"outside 1..L" in engine.hhmm_last_error()
    # a device-pointer request is not range-checked on the host
    assert _validate(engine, pr, host=0) == _abi.OK


def test_validate_rejects_bad_requests(engine):
    pr = _prepared()
    pr.req.abi_version = 99
    assert _validate(engine, pr) == _abi.ERR_INVALID_ARGUMENT
    pr = _prepared()
    pr.req.outputs |= _abi.OUT["oblik_t"]  # not declared by hmm-multinom.stan
    assert _validate(engine, pr) == _abi.ERR_INVALID_ARGUMENT
    pr = _prepared()
    pr.res.gamma_tk = None
    assert _validate(engine, pr) == _abi.ERR_INVALID_ARGUMENT
    pr = _prepared("hhmm-tayal2009")
    pr.req.data.K = 3
    assert _validate(engine, pr) == _abi.ERR_INVALID_ARGUMENT
    pr = _prepared()
    pr.req.pairing = _abi.PAIR_ZIP  # N=2 series vs S=3 draws
    assert _validate(engine, pr) == _abi.ERR_INVALID_ARGUMENT
    assert engine.hhmm_num_pairs(C.byref(pr.req)) == -1


def test_workspace_size_positive(engine):
    pr = _prepared()
    n = C.c_size_t(0)
    assert engine.hhmm_workspace_size(C.byref(pr.req), C.byref(n)) == _abi.OK
    assert n.value > 0


def test_no_cpu_fallback_without_gpu(engine):
    """The product path has no CPU fallback: without a gfx950 device it fails."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    data, draws = synth.hmm_multinom(N=1, S=2, T=5)
    with pytest.raises(api.HHMMError) as e:
        api.gqs("hmm-multinom", data, draws, lib=engine)
    assert e.value.status == _abi.ERR_NO_DEVICE


def test_version_string(engine):
    assert engine.hhmm_version().startswith(b"hhmm-mi355x")


def _source_hash():
    """sha256 over the library's sources in sorted-path order, as the Makefile
    computes it for hhmm_version() (csrc/Makefile SRC_HASH)."""
    import hashlib
    import os
    csrc = REPO / "gsoc17-hhmm_amd" / "csrc"
    rel = [f for f in os.listdir(csrc) if f.endswith((".hip", ".cpp", ".h"))]
    rel += ["../../include/" + f for f in os.listdir(REPO / "include") if f.endswith(".h")]
    rel.append("Makefile")
    h = hashlib.sha256()
    for f in sorted(rel):
        h.update((csrc / f).read_bytes())
    return h.hexdigest()[:16]


def test_library_is_built_from_these_sources(engine):
    """The shipped libhhmm.so names the hash of the sources it was built from;
    it must be this tree's (a stale or foreign build fails here)."""
    v = engine.hhmm_version().decode()
    assert v.split(" src ")[-1] == _source_hash(), (v, _source_hash())


def test_segment_summary_validates_the_request_before_launching(engine):
    """the summary call of a segment window checks the request side
    (draw and data pointers) before any launch, so a NULL draw array is an
    argument error, not a device fault -- reported even without a GPU."""
    from hhmm_amd import segment
    segment.declare(engine)
    pr = _prepared("hmm")
    pr.req.outputs = _abi.OUT["loglik"] | _abi.OUT["gamma_tk"]
    pr.req.data.T = None
    pr.req.draws.A_ij = None
    seg = segment.Segment(1, 1, 0x1000, None, None)
    st = engine.hhmm_segment_summary_device(C.byref(pr.req), C.byref(seg), None, 0, None)
    assert st == _abi.ERR_INVALID_ARGUMENT
    assert b"A_ij" in engine.hhmm_last_error()


def test_python_constants_match_header():
    """Every HHMM_* integer #define / enum value of include/hhmm.h that hhmm_amd._abi
    mirrors has the header's value (status codes, pair status, models, pairing, flags)."""
    import re
    from hhmm_amd import _abi
    text = (REPO / "include" / "hhmm.h").read_text()
    vals = {}
    for name, v in re.findall(r"#define HHMM_(\w+)\s+\(?(\d+)u?\)?\s", text):
        vals[name] = int(v)
    for name, v in re.findall(r"#define HHMM_(\w+)\s+\(1u << (\d+)\)", text):
        vals[name] = 1 << int(v)
    for name, v in re.findall(r"HHMM_(\w+)\s*=\s*(-?\d+)", text):
        vals[name] = int(v)
    checked = 0
    for name, hv in vals.items():
        for py in (name, name.replace("MODEL_", "")):
            if hasattr(_abi, py) and isinstance(getattr(_abi, py), int):
                assert getattr(_abi, py) == hv, (name, getattr(_abi, py), hv)
                checked += 1
                break
    assert _abi.PAIR_INVALID_DATA == vals["PAIR_INVALID_DATA"] == 2
    assert checked >= 15, checked
