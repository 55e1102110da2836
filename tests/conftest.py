import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(autouse=True)
def _log_home(tmp_path, monkeypatch):
    """Apps write training logs to $SPARKNET_HOME; keep them out of the checkout."""
    monkeypatch.setenv("SPARKNET_HOME", str(tmp_path / "logs"))


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sparknet_amd.ops import _lib
    _lib.kernels()
    return torch.device("cuda:0")
