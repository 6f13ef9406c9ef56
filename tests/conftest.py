import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "multiproc: spawns torch.distributed worker processes (gloo)")


def _ensure_native():
    try:
        import flexmi._native  # noqa: F401
        return True
    except ImportError:
        pass
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import build_ext
        build_ext.build(only="native")
        import flexmi._native  # noqa: F401
        return True
    except Exception as e:  # pragma: no cover
        print("native build failed:", e)
        return False


@pytest.fixture(scope="session")
def native():
    assert _ensure_native(), "flexmi._native could not be built"
    import flexmi._native as n
    return n


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import flexmi._C  # noqa: F401  -- fail loudly: GPU tests must run the HIP kernels
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)
