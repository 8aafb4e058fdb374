"""Teardown probe under rocprofv3 (GPU box): what does a process that exits after GPU work need for a
clean exit under a given profiler mode?  --mode torch: torch only (device tensors, a copy, a kernel);
--mode hlc-only: the library without PyTorch (one engine, a page-locked arena, one host-buffer wire call);
--mode hlc: PyTorch and the library (one engine, a page-locked arena, one host-buffer wire call through
the pipelined entry), closed by the library's atexit hook; --mode hlc-close: the same, closed
explicitly before exit.  Prints one line and exits 0; a crash after that line is the teardown's."""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["torch", "hlc-only", "hlc", "hlc-close"], default="hlc")
    a = ap.parse_args()
    import numpy as np
    if a.mode != "hlc-only":
        import torch
        x = torch.arange(1 << 20, device="cuda", dtype=torch.float32)
        y = (x * 2).cpu()
        torch.cuda.synchronize()
    if a.mode == "torch":
        print("torch ok", float(y[-1]), flush=True)
        return 0
    from hashgraph_like_consensus import _ffi, synth
    from hashgraph_like_consensus.engine import Engine
    eng = Engine(0)
    w = synth.generate(64, 16, 16, True, 0x5EED, *synth.engine_signers(eng))
    wire, off, lens, scope = synth.to_wire(w.batch, w.desc)
    arena = _ffi.PinnedArena(wire.size + 64)
    pw = arena.take(wire.shape, np.uint8)
    pw[:] = wire
    res, _, nv = eng.validate_wire_proposals(pw, off, lens, scope, w.now)
    print("hlc ok", int(nv), int(res.shape[0]), flush=True)
    if a.mode == "hlc-close":
        arena.close()
        eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
