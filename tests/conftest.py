"""Shared pytest setup.

* ``-m gpu`` tests need a real MI355X and call the HIP path through the C ABI.
* everything else runs on CPU: the oracle against the golden fixtures, host
  logic (DADA rings, headers, CLIs), the ABI surface of libpafb2p.so (loaded,
  symbols present, no compute), and multi-process gloo tests.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "paf-baseband2power_amd")
ORACLE = os.path.join(REPO, "oracle")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpafb2p.so)")
    config.addinivalue_line("markers", "slow: long-running")


def load_golden(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, f"{name}.npz")) as z:  # allow_pickle=False
        return {k: z[k] for k in z.files}


def golden_geom(d: dict, **over):
    import b2p_oracle as npo
    kw = {k[5:]: int(v) for k, v in d.items() if k.startswith("geom_")}
    kw.update(over)
    return npo.Geom(**kw)


@pytest.fixture(scope="session")
def have_gpu() -> bool:
    import paf_b2p
    return paf_b2p.device_count() > 0


@pytest.fixture
def gpu(have_gpu):
    if not have_gpu:
        pytest.fail("gpu test selected but no HIP device is visible")
    return 0
