import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


_METRICS = {}


def record_metric(name: str, value) -> None:
    """A figure a test measured (e.g. the bit-exact fraction), printed in the session summary even under -q, so it
    reaches the GPU run's log tail."""
    _METRICS[name] = value


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    if _METRICS:
        terminalreporter.write_sep("-", "walker_gym_amd metrics")
        for k, v in _METRICS.items():
            terminalreporter.write_line(f"{k}: {v}")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
