"""Config 3 on one GPU: one P2P proposal of 1,000,000 chained votes, n = 1.5M,
generated on the device; times hlc_validate_proposals_device with the inputs resident in HBM and
reports votes/s, the recovery bracket and the chain-check + tally bracket (global hash tables)."""
import json
import sys
import time

import os  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hashgraph-like-consensus_amd", "python"))
import torch  # noqa: E402

from hashgraph_like_consensus import synth  # noqa: E402
from hashgraph_like_consensus.device import DeviceBatch  # noqa: E402
from hashgraph_like_consensus.engine import Engine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
eng = Engine(0)
t = time.perf_counter()
db = DeviceBatch.synthetic(eng, 1, 1_000_000, 1_500_000, False, synth.config_seed(3), device="cuda:0")
torch.cuda.synchronize()
gen_s = time.perf_counter() - t
eng.reserve(db.n, 1, db.bytes_len)
s = torch.cuda.Stream(device="cuda:0")
eng.validate_proposals_device(db, s.cuda_stream)
torch.cuda.synchronize()
res = db.results_numpy()
assert int(res["status"][0]) == 0 and int(res["total"][0]) == db.n, res
assert (db.status_numpy() == 0).all()
eng.set_kernel_timing(True)
eng.take_kernel_time()
eng.take_chain_time()
t = time.perf_counter()
for _ in range(steps):
    eng.validate_proposals_device(db, s.cuda_stream)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / steps
rec_ms, rec_n, _, _ = eng.take_kernel_time()
ch_ms, ch_n = eng.take_chain_time()
print(json.dumps({"config": "config3: 1 P2P proposal, 1,000,000 chained votes, n = 1,500,000",
                  "votes_per_s": db.n / dt, "ms_per_call": dt * 1e3, "recovery_ms": rec_ms / max(rec_n, 1),
                  "chain_tally_ms": ch_ms / max(ch_n, 1),
                  "chain_tally_GBps": (250 * db.n + 16) / (ch_ms / max(ch_n, 1) / 1e3) / 1e9,
                  "gen_seconds": gen_s}), flush=True)
eng.close()
