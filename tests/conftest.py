import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libcmpc.so")
    config.addinivalue_line("markers", "slow: long-running")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
