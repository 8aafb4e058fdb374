"""Small-batch latency of hlc_eth_verify_batch (GPU box): the batched EthereumConsensusSigner::verify
that the reference calls once per vote (/root/reference/src/utils.rs:154, via process_incoming_vote,
service.rs:293-298).  Host buffers in and out, blocking; per batch size the median wall time of
--reps calls after warm-up, and the per-item time.  Items: random payloads signed by the GPU signer
(hlc_eth_sign_batch), owners from hlc_eth_address_batch; every item must verify Ok(true).

    python tools/verify_latency.py --sizes 1,8,64,1024,65536
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,8,64,1024,65536")
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import numpy as np

    from hashgraph_like_consensus.engine import Engine

    eng = Engine(0)
    sizes = [int(x) for x in a.sizes.split(",")]
    nmax = max(sizes)
    rng = np.random.default_rng(0x484C4339)
    priv = rng.integers(1, 255, size=(nmax, 32), dtype=np.uint8)
    priv[:, 0] = 0x11  # < n
    payloads = [rng.integers(0, 256, size=114, dtype=np.uint8).tobytes() for _ in range(nmax)]
    sigs = eng.sign_batch(priv, payloads)
    owners = eng.address_batch(priv)
    ids = [owners[i].tobytes() for i in range(nmax)]
    sg = [sigs[i].tobytes() for i in range(nmax)]
    for n in sizes:
        st, _ = eng.eth_verify_batch(ids[:n], payloads[:n], sg[:n])
        assert (st == 0).all(), "a signed item did not verify"
        times = []
        reps = a.reps if n <= 4096 else max(3, a.reps // 10)
        for _ in range(reps):
            t = time.perf_counter()
            eng.eth_verify_batch(ids[:n], payloads[:n], sg[:n])
            times.append(time.perf_counter() - t)
        med = statistics.median(times)
        print(json.dumps({"n": n, "median_ms_per_call": med * 1e3, "us_per_item": med / n * 1e6,
                          "items_per_s": n / med, "reps": reps}), flush=True)
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
