"""hlc_eth_verify_batch at the C ABI (GPU box): the batched EthereumConsensusSigner::verify that
the reference calls once per vote (/root/reference/src/signing.rs:69-73, src/utils.rs:154).  Items
are pre-packed into one byte arena with per-item (offset, length) arrays, so the timer holds only the
ABI call: host buffers in (staged and uploaded by the library), statuses and recovered addresses
out, blocking.  Per batch size the median wall time of --reps calls after warm-up.  Items: payloads
of the config-2 vote encoding length (114 B) signed by the GPU signer (hlc_eth_sign_batch), owners
from hlc_eth_address_batch; every item must verify Ok(true) with the signer's address.

    python tools/verify_latency.py --sizes 1,64,1024,65536,640000
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


def pack(ids, payloads, sigs):
    """(arena, id_off, id_len, pay_off, pay_len, sig_off, sig_len): item i's identity, payload and
    signature one after another in the arena (the layout a prost-decoded batch has)."""
    import numpy as np
    n = ids.shape[0]
    rec = ids.shape[1] + payloads.shape[1] + sigs.shape[1]
    arena = np.concatenate([ids, payloads, sigs], axis=1).reshape(-1).copy()
    base = np.arange(n, dtype=np.uint64) * np.uint64(rec)
    id_off, pay_off = base, base + np.uint64(ids.shape[1])
    sig_off = pay_off + np.uint64(payloads.shape[1])
    ln = lambda k: np.full(n, k, np.uint32)  # noqa: E731
    return arena, id_off, ln(ids.shape[1]), pay_off, ln(payloads.shape[1]), sig_off, ln(sigs.shape[1])


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,8,64,1024,16384,65536,262144,640000")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--payload", type=int, default=114)
    a = ap.parse_args()
    import numpy as np

    from hashgraph_like_consensus.engine import Engine

    eng = Engine(0)
    sizes = [int(x) for x in a.sizes.split(",")]
    nmax = max(sizes)
    rng = np.random.default_rng(0x484C4339)
    nkeys = min(nmax, 4096)
    priv = rng.integers(1, 255, size=(nkeys, 32), dtype=np.uint8)
    priv[:, 0] = 0x11  # < n
    owners = eng.address_batch(priv)
    payloads = rng.integers(0, 256, size=(nmax, a.payload), dtype=np.uint8)
    key = np.arange(nmax) % nkeys
    sigs = np.zeros((nmax, 65), np.uint8)
    step = 65536
    for s0 in range(0, nmax, step):  # signing in batches (untimed)
        s1 = min(nmax, s0 + step)
        m = s1 - s0
        arena = np.ascontiguousarray(payloads[s0:s1]).reshape(-1)
        off = np.arange(m, dtype=np.uint64) * np.uint64(a.payload)
        sigs[s0:s1] = eng.sign_batch_arena(np.ascontiguousarray(priv[key[s0:s1]]), arena, off,
                                           np.full(m, a.payload, np.uint32), arena.size)
    ids = owners[key]
    for n in sizes:
        arrs = pack(ids[:n], payloads[:n], sigs[:n])
        st, addr = eng.eth_verify_arrays(*arrs)
        assert (st == 0).all() and np.array_equal(addr, ids[:n]), "a signed item did not verify"
        out = (np.zeros(n, np.uint8), np.zeros((n, 20), np.uint8))
        times = []
        reps = a.reps if n <= 16384 else max(5, a.reps // 5)
        for _ in range(reps):
            t = time.perf_counter()
            eng.eth_verify_arrays(*arrs, out=out)
            times.append(time.perf_counter() - t)
        med = statistics.median(times)
        print(json.dumps({"n": n, "median_ms_per_call": med * 1e3, "us_per_item": med / n * 1e6,
                          "items_per_s": n / med, "reps": reps,
                          "bytes_in_per_call": int(sum(x.nbytes for x in arrs))}), flush=True)
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
