import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kubernetes_gpu_cluster_amd import ops
    ops.load_extension(strict=True)   # GPU tests must exercise the native path
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _kernel_debug_check(request):
    """Under KGC_HIP_DEBUG=1 (the bounds-checking build), fail any GPU test after which
    a K1/K2/K3 device check tripped."""
    yield
    if os.environ.get("KGC_HIP_DEBUG", "0") not in ("", "0") and "gpu" in request.fixturenames:
        from kubernetes_gpu_cluster_amd import ops
        ops.debug_check()
