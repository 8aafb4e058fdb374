#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer entry points: the same config-2 workload
as bench.py, passed as host numpy buffers, so every call stages inputs H2D and results D2H."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"))

from hashgraph_like_consensus import synth  # noqa: E402
from hashgraph_like_consensus.engine import Engine  # noqa: E402


def main() -> None:
    eng = Engine(0)
    addr_fn, sign_fn = synth.engine_signers(eng)
    w = synth.generate(10_000, 64, 64, True, synth.config_seed(2), addr_fn, sign_fn, name="config2")
    wire, off, lens, scope = synth.to_wire(w.batch, w.desc)
    out = {}
    for name, call in (("validate_proposals (host SoA)", lambda: eng.validate_proposals(w.batch, w.desc, w.now,
                                                                                        want_votes=True)),
                       ("validate_wire_proposals (host wire bytes)",
                        lambda: eng.validate_wire_proposals(wire, off, lens, scope, w.now))):
        call()
        t0 = time.perf_counter()
        for _ in range(3):
            res = call()
        dt = (time.perf_counter() - t0) / 3
        assert (res[0]["status"] == 0).all()
        out[name] = {"ms_per_call": dt * 1e3, "votes_per_s": w.batch.n / dt,
                     "bytes_in": int(w.batch.arena.size if "SoA" in name else wire.size)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
