"""Test configuration: import paths for the product package and the oracle, the `gpu` marker."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libhlc.so; run with -m gpu")


@pytest.fixture(scope="session")
def engine():
    from hashgraph_like_consensus.engine import Engine
    # torch (device-memory plumbing of DeviceBatch) must bring up its HIP runtime before libhlc
    # creates a context in this process, as bench.py does
    import torch
    torch.zeros(1, device="cuda:0")
    eng = Engine(0)
    yield eng
    eng.close()
