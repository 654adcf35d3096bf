import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libsiddhi_hip.so)")


def pytest_sessionstart(session):
    # GPU runs mix torch (device buffers) with libsiddhi_hip.so, which loads ROCm's HIP runtime
    # while torch ships its own: torch's must initialise the device first (siddhi_amd.native
    # does the same when torch is already imported).
    if session.config.getoption("-m") and "not gpu" not in session.config.getoption("-m"):
        import torch
        torch.cuda.is_available()
