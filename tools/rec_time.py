"""Time hlc_validate_proposals_device on the config-2 batch with whatever library HLC_LIB names,
without asserting outcomes (for timing-only probe variants whose results are not meaningful).
Prints ms per call, recovery-bracket ms and the fraction of votes the build verified."""
import sys
import time

import os  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hashgraph-like-consensus_amd", "python"))
import torch  # noqa: E402

from hashgraph_like_consensus import synth  # noqa: E402
from hashgraph_like_consensus.device import DeviceBatch  # noqa: E402
from hashgraph_like_consensus.engine import Engine  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "lib"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
eng = Engine(0)
db = DeviceBatch.synthetic(eng, 10_000, 64, 64, True, synth.config_seed(2), start_proposal=0, device="cuda:0")
eng.reserve(db.n, 10_000, db.bytes_len)
s = torch.cuda.Stream(device="cuda:0")
for _ in range(2):
    eng.validate_proposals_device(db, s.cuda_stream)
torch.cuda.synchronize()
eng.set_kernel_timing(True)
eng.take_kernel_time()
t0 = time.perf_counter()
for _ in range(steps):
    eng.validate_proposals_device(db, s.cuda_stream)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
rec_ms, rec_n, _, _ = eng.take_kernel_time()
ok = float((db.status_numpy() == 0).mean())
print(f"{tag} ms_per_call {dt * 1e3:.3f} rec_ms {rec_ms / max(rec_n, 1):.3f} votes_per_s {db.n / dt / 1e6:.1f}M "
      f"verified_frac {ok:.3f}", flush=True)
eng.close()
