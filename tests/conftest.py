import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "isaacgymenvs-ma_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — runs on the GPU box")


def pytest_sessionfinish(session, exitstatus):
    """MIGYM_PARITY_REPORT=<path>: the GPU-vs-oracle error statistics the physics tests recorded"""
    try:
        import parity_stats
    except Exception:  # noqa: BLE001
        return
    parity_stats.write_report()
