import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_sessionstart(session):
    """GPU runs: let torch bring up its HIP runtime before liblo_icp.so does.  The library links the system
    ROCm runtime and torch ships its own; torch's initialisation fails ("No HIP GPUs are available") once the
    other runtime holds the device, and a few GPU tests raycast their synthetic scans with torch (synth.py)."""
    expr = session.config.getoption("-m") or ""
    if "gpu" not in expr or "not gpu" in expr:
        return
    try:
        import torch
        if torch.cuda.is_available():
            torch.zeros(1, device="cuda")
    except Exception:
        pass
