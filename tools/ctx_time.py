"""Time hlc_ctx_create (fixed-base table builds) on the GPU box."""
import sys
import time

sys.path.insert(0, "hashgraph-like-consensus_amd/python")
import torch  # noqa: E402

torch.zeros(1, device="cuda:0")
from hashgraph_like_consensus.engine import Engine  # noqa: E402

for k in range(2):
    t = time.time()
    e = Engine(0)
    print("hlc_ctx_create seconds", round(time.time() - t, 3), flush=True)
    e.close()
