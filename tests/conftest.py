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


@pytest.fixture(autouse=True)
def device_ring_exports_clean():
    """every GPU-resident ring a test makes (paf_b2p.dada.create_ring,
    device >= 0) had each of its blocks exported by the holder at the first
    try: a ring-block export retry fails the test that made the ring.  The
    holder's primer refusal (its first, unused allocation) is
    allowed and counted in the session summary."""
    from paf_b2p import dada
    n0 = len(dada.DEVICE_RINGS)
    yield
    bad = [r for r in dada.DEVICE_RINGS[n0:] if r["export_retries"]]
    assert not bad, f"device-ring block exports retried by the holder: {bad}"


def pytest_terminal_summary(terminalreporter):
    from paf_b2p import dada
    rings = dada.DEVICE_RINGS
    if rings:
        terminalreporter.write_line(
            f"device rings made: {len(rings)}; ring-block export retries: "
            f"{sum(r['export_retries'] for r in rings)}; holder primer refusals: "
            f"{sum(r['primer_refused'] for r in rings)}")
