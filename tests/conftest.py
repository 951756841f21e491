import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libfloam_amd.so")
    config.addinivalue_line("markers", "slow: multi-second CPU test")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def prefilled_map(oracle_lib):
    """prefilled_map(config) -> (edge map, surf map): the raw map initMapWithPoints receives at BASELINE.json's
    config sizes (floam_amd.synth.prefill_map with the oracle's featureExtraction, byte-identical to the GPU's),
    built once per session."""
    from floam_amd import synth
    cache = {}

    def get(config):
        if config not in cache:
            fe = lambda raw, R: oracle_lib.feature_extraction(raw, R, 0.5, 90.0, canonical=True)[:2]
            cache[config] = synth.prefill_map(config, fe)
        return cache[config]
    return get


@pytest.fixture(scope="session")
def floam_gpu():
    """The HIP product path.  GPU tests must never pass on a fallback: fail loudly if the library or device is
    missing."""
    import floam_amd
    from floam_amd import _ffi
    _ffi.load()   # raises if the .so is not built
    c = floam_amd.DeviceCloud()   # raises FloamError(ERR_DEVICE) without a gfx950 device
    c.close()
    return floam_amd
