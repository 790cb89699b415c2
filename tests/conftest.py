"""Shared test setup.

Markers: `gpu` = needs an MI355X (runs through libhhmm.so); everything else
runs on CPU.  The CPU oracle (oracle/) is the checker; it is built on demand.
"""
import pathlib
import sys

import numpy as np
import pytest

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "gsoc17-hhmm_amd"))
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X)")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.load("cr")
    pyoracle.load("libm")
    return pyoracle


@pytest.fixture(scope="session")
def engine():
    import torch  # noqa: F401  (its HIP runtime initialises first: hhmm_amd.api._init_torch_first)
    import hhmm_amd
    return hhmm_amd.load_library()
