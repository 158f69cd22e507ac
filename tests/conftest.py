import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def orc():
    import oracle

    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def golden():
    import json

    d = os.path.join(ROOT, "tests", "golden")
    out = {}
    for name in ["hash", "full", "legacy", "probe"]:
        with open(os.path.join(d, name + ".json")) as f:
            out[name] = json.load(f)
    return out


@pytest.fixture(scope="session")
def gpu():
    """A dlsm_amd context on cuda:0 (GPU tests only)."""
    import torch

    import dlsm_amd

    if not dlsm_amd.device_available():
        pytest.fail("GPU test requested but no HIP device is visible")
    ctx = dlsm_amd.Context(0)
    # one stream for torch's tensor ops and the context: inputs a test makes
    # with torch are ordered before the library's kernels that read them
    s = torch.cuda.Stream(device=0)
    torch.cuda.set_stream(s)
    ctx.set_stream(s)
    yield ctx
    torch.cuda.synchronize()
    ctx.set_stream(None)
    ctx.close()
