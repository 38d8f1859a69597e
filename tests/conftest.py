"""Test configuration: the `gpu` marker and shared scene builders.

`-m "not gpu"` runs here (no GPU): oracle vs reference golden vectors, the dense torch reference
vs the oracle, host logic, C-ABI loading/exports, gloo multi-process tests.
`-m gpu` runs on the MI355X box: HIP path vs oracle parity through the C ABI.
"""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) device")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
