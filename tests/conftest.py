import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


_GPU_WHY = []


def gpu_available():
    try:
        from chanamq_amd import ops
        n = ops.load().device_count()
        if n <= 0:
            _GPU_WHY.append(f"device_count() = {n}")
        return n > 0
    except Exception as e:   # (reported by the fixture)
        _GPU_WHY.append(repr(e))
        return False


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.fail("GPU test requested but no GPU / data-plane extension available: " + "; ".join(_GPU_WHY))
    return True


@pytest.fixture(autouse=True)
def _stop_leftover_brokers():
    """A GPU broker a failed test left running is stopped at its teardown: its native
    threads would otherwise end the process with std::terminate at exit (abort, and the
    GPU run stops there instead of reporting the failure)."""
    yield
    if os.environ.get("CHANAMQ_KEEP_LEFTOVER_BROKERS"):
        return
    mod = sys.modules.get("chanamq_amd.server.gpu_broker")
    live = getattr(getattr(mod, "GpuBroker", None), "_live", None) if mod else None
    for b in list(live or []):
        try:
            b.stop()
        except Exception:   # noqa: BLE001 - best effort
            pass
