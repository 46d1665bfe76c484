import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


def pytest_collection_finish(session):
    """GPU runs: initialise torch's HIP runtime before any test loads libsiddhi_hip.so. torch ships
    its own libamdhip64 / libhsa-runtime64 beside the /opt/rocm ones the engine links, and the second
    runtime to start in a process can fail to find the device once the first has many engines'
    queues open ("No HIP GPUs are available"); torch first is the order bench.py and smoke() use."""
    if any(item.get_closest_marker("gpu") for item in session.items):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:  # noqa: BLE001 -- a CPU-only box: the gpu tests report it themselves
            pass
