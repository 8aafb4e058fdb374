"""hlc_validate_proposals_device at several batch sizes (config-2 shape: P proposals x 64 votes),
10 timed calls each: the per-call fixed cost of the recovery kernels (run under rocprofv3
--kernel-trace for per-kernel times)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hashgraph-like-consensus_amd", "python"))
import torch  # noqa: E402

from hashgraph_like_consensus import synth  # noqa: E402
from hashgraph_like_consensus.device import DeviceBatch  # noqa: E402
from hashgraph_like_consensus.engine import Engine  # noqa: E402

eng = Engine(0)
s = torch.cuda.Stream(device="cuda:0")
for P in [int(x) for x in (sys.argv[1:] or ["2500", "5000", "10000", "20000", "40000"])]:
    db = DeviceBatch.synthetic(eng, P, 64, 64, True, synth.config_seed(2), device="cuda:0")
    eng.reserve(db.n, P, db.bytes_len)
    eng.validate_proposals_device(db, s.cuda_stream)
    torch.cuda.synchronize()
    eng.set_kernel_timing(True)
    eng.take_kernel_time()
    t = time.perf_counter()
    for _ in range(10):
        eng.validate_proposals_device(db, s.cuda_stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 10
    rec_ms, rec_n, _, _ = eng.take_kernel_time()
    eng.set_kernel_timing(False)
    print(f"P {P} votes {db.n} ms_per_call {dt * 1e3:.3f} rec_ms {rec_ms / max(rec_n, 1):.3f} "
          f"Mvotes/s {db.n / dt / 1e6:.1f}", flush=True)
    del db
    torch.cuda.empty_cache()
eng.close()
