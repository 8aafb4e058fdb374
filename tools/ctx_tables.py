"""Context creation with the per-device fixed-base tables (hlc_api.cpp gen_tables): the first context on
a device builds them, later ones share them; a context created after all others were destroyed builds
them again.  Prints the wall time of each step and the device memory in use (GPU box)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"))
import torch  # noqa: E402
from hashgraph_like_consensus.engine import Engine  # noqa: E402


def used_gb():
    free, total = torch.cuda.mem_get_info(0)
    return (total - free) / 1e9


def timed(label, fn):
    t = time.perf_counter()
    r = fn()
    print(f"{label:34s} {1e3 * (time.perf_counter() - t):8.1f} ms   device memory in use {used_gb():6.2f} GB",
          flush=True)
    return r


torch.cuda.init()
print(f"{'before any context':34s} {'':8s}      device memory in use {used_gb():6.2f} GB")
a = timed("first context (builds the tables)", Engine)
b = timed("second context (shares them)", Engine)
c = timed("third context", Engine)
timed("destroy all three", lambda: [e.close() for e in (a, b, c)])
d = timed("new context (builds them again)", Engine)
d.close()
