import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
SCENES = os.path.join(ROOT, "scenes")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle():
    from oracle_lib import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def rt():
    """The product library; GPU tests require a device (no fallback)."""
    import torch  # noqa: F401  -- first, so torch and librt_amd.so bind the same HIP runtime
    import rtamd
    rtamd.lib()
    return rtamd


@pytest.fixture(scope="session")
def gpu(rt):
    n = rt.device_count()
    assert n >= 1, "GPU test without a HIP device"
    return rt


def scene_path(name):
    return os.path.join(SCENES, name + ".json")
