import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libsiddhi_hip.so)")


def pytest_collection_modifyitems(session, config, items):
    # GPU runs mix torch (device buffers) with libsiddhi_hip.so, which loads ROCm's HIP runtime
    # while torch ships its own: torch's must initialise the device first (siddhi_amd.native
    # does the same when torch is already imported).  Any selected GPU test (by -m or -k)
    # triggers it before the first test runs.
    if any(item.get_closest_marker("gpu") for item in items):
        import torch
        if torch.cuda.is_available():
            torch.zeros(1, device="cuda")
